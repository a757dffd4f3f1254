"""Shared bearer token between the node agent and the culler.

The node agent listens on a hostPort, so anything that can reach the node can reach it.
Its data endpoints (``/gpu/*``, ``/metrics``) list pod UIDs and names with their GPUs and
VRAM.  When a token file is configured, those endpoints answer only requests that carry
``Authorization: Bearer <token>``.  ``/healthz`` stays open for the kubelet's probe.

The token lives in a Secret (``mi355x-node-agent-token``, written by
``cmd/webhook_certs --random-secret``, or by an admin) that both the DaemonSet and the kf
manager mount.  The file is re-read when its mtime changes, because the kubelet updates
mounted Secrets in place, so a rotated token takes effect without a restart.  A configured
but missing or empty file fails closed: every data request is refused until it appears.
"""

from __future__ import annotations

import hmac
import os
import time
from typing import Optional

TOKEN_SECRET = "mi355x-node-agent-token"
TOKEN_KEY = "token"
TOKEN_MOUNT = "/var/run/secrets/odh/node-agent"


class TokenFile:
    """A token file, re-read when it changes (checked at most every ``recheck_s`` seconds)."""

    def __init__(self, path: str, recheck_s: float = 1.0):
        self.path = path
        self.recheck_s = recheck_s
        self._token: Optional[str] = None
        self._stamp = None
        self._checked = -1e18

    def current(self) -> Optional[str]:
        now = time.monotonic()
        if now - self._checked < self.recheck_s:
            return self._token
        self._checked = now
        try:
            st = os.stat(self.path)
        except OSError:
            self._token, self._stamp = None, None
            return None
        stamp = (st.st_mtime_ns, st.st_size, st.st_ino)
        if stamp != self._stamp:
            try:
                with open(self.path) as f:
                    tok = f.read().strip()
            except OSError:
                tok = ""
            self._token, self._stamp = (tok or None), stamp
        return self._token

    def authorizes(self, header: Optional[str]) -> bool:
        """True when ``header`` is ``Bearer <the current token>``.  No token: False."""
        tok = self.current()
        if not tok or not header or not header.startswith("Bearer "):
            return False
        return hmac.compare_digest(header[7:].strip().encode(), tok.encode())

    def header(self) -> dict:
        """The request header the client side sends (empty while no token is readable)."""
        tok = self.current()
        return {"Authorization": f"Bearer {tok}"} if tok else {}


async def ensure_token_secret(client, namespace: str, name: str = TOKEN_SECRET, key: str = TOKEN_KEY) -> str:
    """Create Secret ``name`` holding a random token if it does not exist (idempotent: an
    existing, non-empty token is kept, so re-running the provisioner never rotates it under the
    running agents).  Returns ``"created"``, ``"kept"`` or ``"filled"`` (existed without the key)."""
    import base64
    import secrets

    from ..models import kinds
    from ..models.errors import ApiError, is_not_found

    tok = base64.b64encode(secrets.token_urlsafe(32).encode()).decode()
    try:
        cur = await client.get(kinds.SECRET, name, namespace)
    except ApiError as e:
        if not is_not_found(e):
            raise
        await client.create({"apiVersion": "v1", "kind": "Secret", "type": "Opaque",
                             "metadata": {"name": name, "namespace": namespace,
                                          "labels": {"app.kubernetes.io/managed-by": "odh-webhook-certs"}},
                             "data": {key: tok}})
        return "created"
    if base64.b64decode((cur.get("data") or {}).get(key) or "").strip():
        return "kept"
    cur.setdefault("data", {})[key] = tok
    await client.update(cur)
    return "filled"
