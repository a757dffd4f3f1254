"""Client interfaces (the ``client.Client`` / ``client.Reader`` analogues) and the cached
client every manager writes through.  (The in-process implementation over the test
platform's object store lives in :mod:`odh_kubeflow_amd.testing.apiserver.inprocess`.)

Two access paths, as in controller-runtime:

* :class:`Reader` — synchronous, read-only, zero-copy reads from the cache.  Event map
  functions and predicates use it (e.g. ``predNBEvents`` at
  ``kf/controllers/notebook_controller.go:755-775`` does a Pod and a Notebook GET per
  event).
* :class:`Client` — async CRUD.  Reads go through the cache unless the kind is listed in
  ``uncached`` (the odh manager disables the cache for ConfigMaps and Secrets,
  ``odh/main.go:178-185``).  Like controller-runtime, write calls refresh the caller's
  object in place with the server response (new ``resourceVersion`` etc.).
"""

from __future__ import annotations

import abc
import asyncio
import contextvars
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Tuple

from ..models.errors import ApiError, is_not_found
from ..models.scheme import SCHEME
from ..utils.objutil import deepcopy_json

WatchCallback = Callable[[str, dict, Optional[dict]], None]


# Set by ``retry_on_conflict`` for its retries: a Conflict means the informer copy is
# stale, so the retry reads through to the apiserver instead of sleeping for the cache.
LIVE_READS: contextvars.ContextVar = contextvars.ContextVar("live_reads", default=False)
# (controller name, request) of the reconcile running in this task, set by the controller's
# worker: writes made under it are remembered so their own watch echo does not queue the
# same request again (see CachedClient.own_write)
CURRENT_RECONCILE: contextvars.ContextVar = contextvars.ContextVar("current_reconcile", default=None)
# Set while an admission webhook handles a request: a one-shot decision with no requeue, so
# an object absent from the informer is confirmed with the apiserver (the reference's live
# read, which sees an object created a moment before the admission) instead of being
# answered NotFound from the cache (see CachedClient._validated)
# (the value: the keys already confirmed absent during this admission, read once)
CONFIRM_ABSENCE: contextvars.ContextVar = contextvars.ContextVar("confirm_absence", default=None)
_RETRY = object()  # a coalesced live read whose sender was cancelled: read again


async def get_live(client, kind, name: str, namespace: Optional[str] = None):
    """``client.get`` straight from the apiserver, whatever the client's cache says — e.g. after a
    create answered AlreadyExists for an object the (data-stripped) informer had not shown yet."""
    tok = LIVE_READS.set(True)
    try:
        return await client.get(kind, name, namespace)
    finally:
        LIVE_READS.reset(tok)
# how long a read of an object this client just wrote waits for the watch to deliver the
# write before it reads through to the apiserver instead
RYOW_WAIT_S = 0.05


def _patch_certainly_changes(patch: Any, patch_type: str, out: Any) -> bool:
    """Whether a successful patch certainly produced a new version (so the answered version
    is this client's own): a resourceVersion precondition that the answer moved past, or a
    JSON patch that removes or changes a value it tested first.  Anything else may have been
    a no-op, answered with whatever version was live."""
    if patch_type == "json" and isinstance(patch, list):
        tested = {}
        for op in patch:
            if not isinstance(op, dict):
                continue
            path, kind = op.get("path"), op.get("op")
            if kind == "test":
                if path == "/metadata/resourceVersion":
                    return str(op.get("value")) != str(((out or {}).get("metadata") or {}).get("resourceVersion"))
                tested[path] = op.get("value")
            elif path in tested and (kind == "remove" or (kind in ("replace", "add") and op.get("value") != tested[path])):
                return True
        return False
    if isinstance(patch, dict):
        want = (patch.get("metadata") or {}).get("resourceVersion") if isinstance(patch.get("metadata"), dict) else None
        if want:
            return str(want) != str(((out or {}).get("metadata") or {}).get("resourceVersion"))
    return False


def _rv_int(o) -> Optional[int]:
    try:
        return int((o.get("metadata") or {}).get("resourceVersion") or "")
    except (TypeError, ValueError, AttributeError):
        return None


def _version_of(ref) -> Optional[str]:
    if isinstance(ref, str):
        api_version = ref.rpartition("/")[0]
        return api_version.rpartition("/")[2] if api_version else None
    if isinstance(ref, dict):
        return ref.get("apiVersion", "").rpartition("/")[2] or None
    return None


def _refresh(target: Optional[dict], new: dict) -> dict:
    if isinstance(target, dict) and target is not new:
        target.clear()
        target.update(new)
        return target
    return new


class Reader(abc.ABC):
    """Synchronous cache reader; returned objects are shared and MUST NOT be mutated."""

    @abc.abstractmethod
    def get(self, kind, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        ...

    @abc.abstractmethod
    def list(self, kind, namespace: Optional[str] = None, labels=None, fields: Optional[str] = None,
             owner_uid: Optional[str] = None) -> List[dict]:
        ...


class EventSource(abc.ABC):
    """Watch subscription provider for controllers (store or informer backed)."""

    @abc.abstractmethod
    def subscribe(self, kind, callback: WatchCallback, namespace: Optional[str] = None) -> Callable[[], None]:
        ...

    async def wait_synced(self, kinds: Iterable) -> None:  # pragma: no cover - trivial default
        return None


class Client(abc.ABC):
    scheme = SCHEME

    @abc.abstractmethod
    async def get(self, kind, name: str, namespace: Optional[str] = None) -> dict:
        ...

    @abc.abstractmethod
    async def list(self, kind, namespace: Optional[str] = None, labels=None, fields: Optional[str] = None,
                   owner_uid: Optional[str] = None) -> List[dict]:
        ...

    @abc.abstractmethod
    async def create(self, obj: dict) -> dict:
        ...

    @abc.abstractmethod
    async def update(self, obj: dict) -> dict:
        ...

    @abc.abstractmethod
    async def update_status(self, obj: dict) -> dict:
        ...

    @abc.abstractmethod
    async def patch(self, obj_or_kind, patch: Any, patch_type: str = "merge", name: Optional[str] = None,
                    namespace: Optional[str] = None, subresource: Optional[str] = None) -> dict:
        ...

    @abc.abstractmethod
    async def delete(self, obj_or_kind, name: Optional[str] = None, namespace: Optional[str] = None,
                     preconditions: Optional[dict] = None, propagation: str = "Background") -> Optional[dict]:
        ...

    async def get_or_none(self, kind, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        from ..models.errors import is_not_found

        try:
            return await self.get(kind, name, namespace)
        except Exception as e:
            if is_not_found(e):
                return None
            raise


async def any_readonly(client, kind, namespace, pred) -> bool:
    """Whether some object of ``kind`` in ``namespace`` satisfies ``pred``: from the cache with
    an early exit when the client has one (``CachedClient.any_readonly``), else over a list."""
    fn = getattr(client, "any_readonly", None)
    if fn is not None:
        return await fn(kind, namespace, pred)
    return any(pred(o) for o in await client.list(kind, namespace))


class CachedClient(Client):
    """Reads from a :class:`Reader` (copying), writes through a backing client.

    Kinds in ``uncached`` are read live from the backing client, exactly like
    ``client.CacheOptions.DisableFor``.

    Unlike controller-runtime's client, reads are consistent with this client's own
    writes: every write records the resourceVersion it produced, and a cached read that
    is older than that (the watch event is still in flight) goes to the apiserver
    instead.  Without it a reconcile triggered between a write and its watch event acts
    on the pre-write object and repeats the write (observed: the odh lock removal patch
    and its admission call issued twice per notebook).
    """

    def __init__(self, reader: Reader, writer: Client, uncached: Sequence = ()):
        self.reader = reader
        self.writer = writer
        self.uncached = {SCHEME.resolve(k).key for k in uncached}
        self._written: Dict[Tuple[str, str, str], int] = {}
        self._ensured: set = set()  # kinds whose informer is known synced and served
        # (kind, namespace, name, resourceVersion) → (controller, request) that wrote it
        self._own: Dict[Tuple[str, str, str, int], tuple] = {}
        # (kind, namespace, name) → [(controller, request), precondition rv or None, the rv of
        # the event provisionally claimed as its echo] of a create / precondition update still
        # awaiting its response (the watch event can overtake the response)
        self._inflight: Dict[Tuple[str, str, str], list] = {}
        # (controller name, request) → re-queue it: set by the manager; called when an event
        # claimed as an in-flight write's echo turns out not to be (see own_write)
        self.requeue: Optional[Callable[[str, Any], None]] = None
        self.misclaims = 0
        self.fresh_reads = 0
        self.cache_waits = 0
        # live-read kinds (``uncached``: the odh manager's ConfigMaps / Secrets, whose cached
        # copies are stripped of their data): key → (resourceVersion, full object) of the
        # last live read or own write, reused while the stripped informer still shows that
        # resourceVersion (see :meth:`_validated`)
        self._full: Dict[Tuple[str, str, str], Tuple[int, dict]] = {}
        self.validated_reads = 0
        # live reads of the same object coalesced (see _live_get): key → (start, future) of the
        # read in flight, and the future of the read that follows it
        self._flight: Dict[Tuple[str, str, str], Tuple[float, asyncio.Future]] = {}
        self._next_flight: Dict[Tuple[str, str, str], asyncio.Future] = {}
        self.coalesced_reads = 0

    def _note(self, out, claim: bool = True) -> None:
        """Remember a write's result.  ``claim=False``: the write may have been a no-op — a
        status patch or a patch without any precondition, which the apiserver answers with
        the live object unchanged, i.e. with SOMEONE ELSE's latest version — so the version
        is not claimed as this controller's echo (claiming it hid the odh lock removal from
        the kf reconciler that had just re-written an unchanged status: the notebook stayed
        at 0 replicas, tests/test_fault_injection.py)."""
        if not isinstance(out, dict) or "metadata" not in out:
            return
        rv = _rv_int(out)
        if rv is None:
            return
        try:
            key = (SCHEME.resolve(out).key, out["metadata"].get("namespace") or "", out["metadata"].get("name", ""))
        except Exception:
            return
        if len(self._written) > 16384:
            self._written.clear()
        self._written[key] = rv
        if key[0] in self.uncached:
            self._keep_full(key, rv, out)
        cur = CURRENT_RECONCILE.get()
        if cur is not None and claim:
            if len(self._own) > 16384:
                self._own.clear()  # echoes never delivered (kinds nobody here watches)
            self._own[key + (rv,)] = cur

    def own_write(self, obj: dict, controller: str):
        """The request whose reconcile in ``controller`` produced exactly this object version
        (its watch echo), else None.  That reconcile already acted on the state it wrote, so
        the echo need not queue the request again — the informer-side counterpart of the
        ``expectations`` kube-controller-manager's controllers keep for their own writes.
        Only an identical resourceVersion matches: any later change by anyone is a new
        event, and other controllers watching the object still see the echo."""
        if not self._own and not self._inflight:
            return None
        rv = _rv_int(obj)
        if rv is None:
            return None
        md = obj.get("metadata") or {}
        try:
            key = (SCHEME.resolve(obj).key, md.get("namespace") or "", md.get("name", ""), rv)
        except Exception:
            return None
        hit = self._own.get(key)
        if hit is None and self._inflight:
            # The echo overtook the write's response.  Only creates and resourceVersion-
            # preconditioned updates are tracked in flight, and only the first event after
            # the precondition is claimed: a write by another client before ours would have
            # failed ours (AlreadyExists / Conflict).  The claim is provisional — a write of
            # someone else can follow ours inside the window, and a preconditioned update can
            # be a no-op — and is settled against the response (_settle).
            ent = self._inflight.get(key[:3])
            if ent is not None:
                if ent[2] is None and (ent[1] is None or rv > ent[1]):
                    ent[2] = rv
                if ent[2] == rv:
                    hit = ent[0]
        # kept (not popped): a controller may watch the kind twice (Owns + Watches); the
        # table is bounded and an entry can only ever match its own object version
        return hit[1] if hit is not None and hit[0] == controller else None

    def _live(self, kind, namespace: Optional[str] = None) -> bool:
        if SCHEME.resolve(kind).key in self.uncached:
            return True
        # a namespace outside a namespace-restricted (sharded) cache is read live: the
        # webhook admits objects of every namespace, whichever shard owns them
        covers = getattr(self.reader, "covers", None)
        return covers is not None and namespace is not None and not covers(kind, namespace)

    async def _ensure(self, kind) -> None:
        if type(kind) is str and kind in self._ensured:
            return
        ensure = getattr(self.reader, "ensure_informer", None)
        if ensure is not None:
            await ensure(kind)  # raises NoKindMatch while the kind is not served
        if type(kind) is str:
            self._ensured.add(kind)

    FULL_CAP = 4096  # objects kept for validated reads (the few ConfigMaps a manager reads)

    def _keep_full(self, key: Tuple[str, str, str], rv: int, obj: dict) -> None:
        if len(self._full) >= self.FULL_CAP:
            self._full.pop(next(iter(self._full)))  # oldest first
        self._full[key] = (rv, deepcopy_json(obj))

    def _validated(self, kind, name: str, namespace: Optional[str]) -> Optional[dict]:
        """A live-read kind's object without the read, when it provably has not changed.

        The reference reads ConfigMaps and Secrets live (``DisableFor``) because its cache
        strips their data (``odh/main.go:81-101,165-185``) — and so does this one.  But the
        stripped informer still carries each object's resourceVersion: when it equals the
        version of the copy this client last read or wrote, the data is that copy's.  So a
        read costs a round trip only after the object changed (or before the informer has
        it) — the unsharded odh manager re-read ``pipeline-runtime-images`` and the CA
        bundles live 16+ times per notebook, mostly to learn they do not exist.  An object
        the synced informer does not hold is NotFound without a read, unless this client
        wrote it or an admission is being decided (``CONFIRM_ABSENCE``: the webhook must see
        a ConfigMap created a moment before, as the reference's live read does; its
        existence-only decisions are safe on a vouched-for copy).  Freshness is the informer's, as for every other cached read; this client's
        own newer writes always win (``_written``)."""
        info = SCHEME.resolve(kind)
        key = (info.key, namespace or "", name)
        watching = getattr(self.reader, "watching", None)
        if watching is None or not watching(kind, namespace):
            return None
        o = self.reader.get(kind, name, namespace)
        if o is None:
            if key in self._written or CONFIRM_ABSENCE.get() is not None:
                # written here and not yet in the cache, or an admission: read through
                return None
            # absent from a synced informer: NotFound, as a cached read would say (the
            # optional bundles — odh-trusted-ca-bundle, pipeline-runtime-images — usually are)
            from ..models.errors import NotFound

            self.validated_reads += 1
            raise NotFound(info.plural if not info.group else f"{info.plural}.{info.group}", name)
        ent = self._full.get(key)
        if ent is None or _rv_int(o) != ent[0]:
            return None
        want = self._written.get(key)
        if want is not None and want > ent[0]:
            return None
        self.validated_reads += 1
        out = deepcopy_json(ent[1])
        v = _version_of(kind)
        if v:
            out["apiVersion"] = info.api_version(v)
        return out

    async def _live_get(self, key, kind, name, namespace):
        """A live GET whose answer is as fresh as a GET issued now would be, coalesced with
        the concurrent live reads of the same object.

        A read may share another's answer only if that GET was sent after this read began (so
        it reflects every write that completed before this read began — what a live read is
        for, e.g. an admission seeing a ConfigMap created a moment before).  A read arriving
        while a GET of the key is in flight therefore waits for the NEXT GET, which is sent
        when the current one answers and serves every read that arrived meanwhile: at most one
        GET per object in flight and one queued, however many admissions of one namespace
        arrive at once (a burst of 64 notebooks read the same two ConfigMaps 128 times).  A
        single read waits for nothing."""
        loop = asyncio.get_running_loop()
        cur = self._flight.get(key)
        if cur is None:
            return deepcopy_json(await self._fly(key, kind, name, namespace))
        nxt = self._next_flight.get(key)
        if nxt is None:
            nxt = self._next_flight[key] = loop.create_future()
        else:
            self.coalesced_reads += 1
        try:
            await asyncio.shield(cur[1])
        except Exception:  # noqa: BLE001 — the current read's outcome is not ours
            pass  # (a cancellation of THIS reader propagates: another waiter sends the next GET)
        if self._next_flight.get(key) is nxt:
            # the first waiter sends the next GET for everyone queued behind the last one
            del self._next_flight[key]
            try:
                o = await self._fly(key, kind, name, namespace)
            except asyncio.CancelledError:
                if not nxt.done():
                    nxt.set_result(_RETRY)  # this reader was cancelled, not the others: they read again
                raise
            except BaseException as e:
                if not nxt.done():
                    nxt.set_exception(e)
                    nxt.exception()  # retrieved: a waiter-less failure is not "never retrieved"
                raise
            if not nxt.done():
                nxt.set_result(o)
            return deepcopy_json(o)
        o = await asyncio.shield(nxt)
        if o is _RETRY:
            return await self._live_get(key, kind, name, namespace)
        return deepcopy_json(o)

    async def _fly(self, key, kind, name, namespace):
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        self._flight[key] = (loop.time(), fut)
        try:
            o = await self.writer.get(kind, name, namespace)
        except BaseException as e:
            if not fut.done():
                fut.set_exception(e)
                fut.exception()
            raise
        finally:
            if self._flight.get(key, (None, None))[1] is fut:
                del self._flight[key]
        fut.set_result(o)
        return o

    async def prefetch(self, keys: Sequence[Tuple[Any, str, Optional[str]]]) -> None:
        """Inside an admission (``CONFIRM_ABSENCE`` set): make the live reads of ``keys`` —
        (kind, name, namespace) that the admission is about to read — concurrently, so that
        confirming N absences costs one round trip instead of N in sequence.  The answers land
        where ``get`` looks first (the validated-read cache, the admission's absence memo)."""
        if CONFIRM_ABSENCE.get() is None or len(keys) < 2:
            return

        async def one(kind, name, namespace):
            try:
                await self.get(kind, name, namespace)
            except ApiError:
                pass  # recorded (NotFound) or raised again by the read itself

        await asyncio.gather(*(one(*k) for k in keys))

    async def get(self, kind, name, namespace=None):
        if self._live(kind, namespace) or LIVE_READS.get():
            uncached = SCHEME.resolve(kind).key in self.uncached
            key = (SCHEME.resolve(kind).key, namespace or "", name)
            absent = CONFIRM_ABSENCE.get() if uncached else None
            if uncached and not LIVE_READS.get():
                hit = self._validated(kind, name, namespace)
                if hit is not None:
                    return hit
                if absent is not None and key in absent and key not in self._written:
                    from ..models.errors import NotFound  # confirmed earlier in this admission

                    info = SCHEME.resolve(kind)
                    raise NotFound(info.plural if not info.group else f"{info.plural}.{info.group}", name)
            try:
                o = await self._live_get(key, kind, name, namespace)
            except ApiError as e:
                if absent is not None and is_not_found(e):
                    absent.add(key)
                raise
            if uncached:
                rv = _rv_int(o)
                if rv is not None:
                    self._keep_full(key, rv, o)
            return o
        await self._ensure(kind)
        o = self.reader.get(kind, name, namespace)
        if self._written:
            key = (SCHEME.resolve(kind).key, namespace or "", name)
            want = self._written.get(key)
            if want is not None:
                have = _rv_int(o) if o is not None else None
                if have is None or have < want:
                    # the cache has not seen our own write yet: let the watch event (already
                    # on its way) land, and read through only if it does not come promptly
                    wait = getattr(self.reader, "wait_for_rv", None)
                    if wait is not None and await wait(kind, namespace, want, RYOW_WAIT_S):
                        self.cache_waits += 1
                        o = self.reader.get(kind, name, namespace)
                        have = _rv_int(o) if o is not None else None
                        if o is not None and have < want:
                            o = None
                            have = None
                        elif o is None:
                            have = want  # deleted after our write: NotFound below is current
                    if have is None or have < want:
                        self.fresh_reads += 1
                        return await self.writer.get(kind, name, namespace)
                del self._written[key]
        if o is None:
            from ..models.errors import NotFound

            info = SCHEME.resolve(kind)
            raise NotFound(info.plural if not info.group else f"{info.plural}.{info.group}", name)
        o = deepcopy_json(o)
        v = _version_of(kind)
        if v:
            o["apiVersion"] = SCHEME.resolve(kind).api_version(v)
        return o

    async def list(self, kind, namespace=None, labels=None, fields=None, owner_uid=None):
        if self._live(kind, namespace) and owner_uid is None:
            return await self.writer.list(kind, namespace, labels, fields)
        await self._ensure(kind)
        items = [deepcopy_json(o) for o in self.reader.list(kind, namespace, labels, fields, owner_uid)]
        v = _version_of(kind)
        if v:
            av = SCHEME.resolve(kind).api_version(v)
            for o in items:
                o["apiVersion"] = av
        return items

    async def any_readonly(self, kind, namespace, pred) -> bool:
        """:func:`any_readonly` on this client's cache (objects shared: ``pred`` must not mutate)."""
        if self._live(kind, namespace):
            return any(pred(o) for o in await self.writer.list(kind, namespace))
        await self._ensure(kind)
        scan = getattr(self.reader, "any", None)
        if scan is not None:
            return scan(kind, namespace, pred)
        return any(pred(o) for o in self.reader.list(kind, namespace))

    def _begin(self, obj, precondition: Optional[int] = None, name: Optional[str] = None,
               namespace: Optional[str] = None) -> Optional[Tuple[str, str, str]]:
        """Track a create / preconditioned write in flight (``obj``: the object, or its kind
        with ``name`` / ``namespace`` — a patch)."""
        cur = CURRENT_RECONCILE.get()
        if cur is None:
            return None
        md = (obj.get("metadata") or {}) if isinstance(obj, dict) else {}
        name = name or md.get("name")
        if not name:
            return None  # generateName: the key is unknown until the response
        try:
            key = (SCHEME.resolve(obj).key, namespace or md.get("namespace") or "", name)
        except Exception:
            return None
        self._inflight[key] = [cur, precondition, None]
        return key

    def _settle(self, key, out) -> None:
        """The write answered (``out``) or failed (None): an event claimed in flight that is
        not this write's version goes back to its controller's queue."""
        ent = self._inflight.pop(key, None)
        if ent is None or ent[2] is None:
            return
        if out is None or _rv_int(out) != ent[2]:
            self.misclaims += 1
            if self.requeue is not None:
                self.requeue(ent[0][0], ent[0][1])

    async def create(self, obj):
        key = self._begin(obj)
        out = None
        try:
            out = await self.writer.create(obj)
        finally:
            if key is not None:
                self._settle(key, out)
        self._note(out)
        return out

    async def update(self, obj):
        sent = _rv_int(obj)
        key = self._begin(obj, sent) if sent is not None else None
        out = None
        try:
            out = await self.writer.update(obj)
        finally:
            if key is not None:
                self._settle(key, out)
        # without a precondition, or answered with the version sent, the update was a no-op
        self._note(out, claim=sent is not None and _rv_int(out) != sent)
        return out

    async def update_status(self, obj):
        sent = _rv_int(obj)
        out = await self.writer.update_status(obj)
        self._note(out, claim=sent is not None and _rv_int(out) != sent)
        return out

    async def patch(self, obj_or_kind, patch, patch_type="merge", name=None, namespace=None, subresource=None):
        # a resourceVersion-preconditioned merge patch is tracked in flight like a
        # preconditioned update: its watch echo can overtake the response (the culler's
        # heartbeat, once per check of every notebook, would otherwise requeue itself)
        key = None
        if subresource is None and patch_type == "merge" and isinstance(patch, dict):
            sent = _rv_int(patch)
            if sent is not None:
                key = self._begin(obj_or_kind, sent, name, namespace)
        out = None
        try:
            out = await self.writer.patch(obj_or_kind, patch, patch_type, name, namespace, subresource)
        finally:
            if key is not None:
                self._settle(key, out)
        self._note(out, claim=_patch_certainly_changes(patch, patch_type, out))
        return out

    async def delete(self, obj_or_kind, name=None, namespace=None, preconditions=None, propagation="Background"):
        if self._written:
            try:
                md = obj_or_kind.get("metadata", {}) if isinstance(obj_or_kind, dict) else {}
                self._written.pop((SCHEME.resolve(obj_or_kind).key, namespace or md.get("namespace") or "",
                                   name or md.get("name", "")), None)
            except Exception:
                pass
        return await self.writer.delete(obj_or_kind, name, namespace, preconditions, propagation)
