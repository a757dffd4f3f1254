"""A TLS server context that follows its certificate files (controller-runtime's
``certwatcher``): the admission webhook and the MI355X node agent serve from a mounted Secret
(``tls.crt`` / ``tls.key``) that a renewal rotates in place; :meth:`ServingCert.maybe_reload`
loads a changed pair into the live context, so new connections present the new certificate
without a restart.  A half-written or mismatched pair is ignored and retried; the old
certificate keeps serving."""

from __future__ import annotations

import asyncio
import logging
import os
import shutil
import ssl
import tempfile
from typing import Optional, Tuple

log = logging.getLogger("tls")


class ServingCert:
    def __init__(self, cert_dir: str, what: str = "serving"):
        self.cert_dir = cert_dir
        self.what = what
        self.ctx: Optional[ssl.SSLContext] = None
        self._stamp: Optional[Tuple] = None
        self.reloads = 0
        self._watch: Optional[asyncio.Task] = None

    def files(self) -> Tuple[str, str]:
        return os.path.join(self.cert_dir, "tls.crt"), os.path.join(self.cert_dir, "tls.key")

    def _file_stamp(self) -> Optional[Tuple]:
        try:
            return tuple((st.st_mtime_ns, st.st_size, st.st_ino) for st in map(os.stat, self.files()))
        except OSError:
            return None

    def context(self) -> ssl.SSLContext:
        ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
        ctx.minimum_version = ssl.TLSVersion.TLSv1_2
        self._stamp = self._file_stamp()
        ctx.load_cert_chain(*self.files())
        self.ctx = ctx
        return ctx

    def maybe_reload(self) -> bool:
        """Load rotated cert files into the live context; True when a new pair was loaded."""
        if self.ctx is None:
            return False
        stamp = self._file_stamp()
        if stamp is None or stamp == self._stamp:
            return False
        # snapshot the pair, prove it on a scratch context, only then load it into the live one:
        # a failed load_cert_chain leaves an SSL_CTX with the new cert and the old key
        with tempfile.TemporaryDirectory(prefix="odh-tls-reload-") as d:
            try:
                crt, key = (shutil.copy(f, os.path.join(d, os.path.basename(f))) for f in self.files())
                scratch = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
                scratch.load_cert_chain(crt, key)
                self.ctx.load_cert_chain(crt, key)
            except (ssl.SSLError, OSError) as e:  # mid-rotation: keep serving the old pair, retry next tick
                log.warning("%s certificate reload failed (old certificate kept): %r", self.what, e)
                return False
        self._stamp = stamp
        self.reloads += 1
        log.info("%s certificate reloaded from %s", self.what, self.cert_dir)
        return True

    def watch(self, interval: float) -> None:
        """Poll the files every ``interval`` seconds (on the running loop) until :meth:`stop`."""
        async def loop():
            while True:
                await asyncio.sleep(interval)
                self.maybe_reload()
        if interval > 0 and self._watch is None:
            self._watch = asyncio.ensure_future(loop())

    def stop(self) -> None:
        if self._watch is not None:
            self._watch.cancel()
            self._watch = None


def client_context(ca_file: str) -> ssl.SSLContext:
    """Verifying client context trusting only ``ca_file`` (hostname checked against the
    certificate's SANs)."""
    ctx = ssl.create_default_context(ssl.Purpose.SERVER_AUTH, cafile=ca_file)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    return ctx
