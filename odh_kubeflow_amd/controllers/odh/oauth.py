"""Legacy OAuthClient cleanup (reference ``odh/controllers/notebook_oauth.go``).

Workbenches of older releases own a cluster-scoped ``OAuthClient``
``<name>-<ns>-oauth-client`` guarded by finalizer
``notebook-oauth-client-finalizer.opendatahub.io``; on deletion it is removed and the
finalizer dropped.  Nothing new is ever created.
"""

from __future__ import annotations

from ...models import kinds
from ...models import meta as m
from ...models.errors import ApiError, is_no_match, is_not_found
from .constants import OAUTH_CLIENT_FINALIZER


def has_oauth_client_finalizer(nb: dict) -> bool:
    return OAUTH_CLIENT_FINALIZER in m.finalizers(nb)


def oauth_client_name(nb: dict) -> str:
    return f"{m.name(nb)}-{m.namespace(nb)}-oauth-client"


async def delete_oauth_client(client, nb: dict) -> None:
    try:
        await client.delete(kinds.OAUTH_CLIENT, oauth_client_name(nb))
    except ApiError as e:
        if not (is_not_found(e) or is_no_match(e)):
            raise


async def remove_oauth_client_finalizer(client, nb: dict) -> None:
    if m.remove_finalizer(nb, OAUTH_CLIENT_FINALIZER):
        await client.update(nb)
