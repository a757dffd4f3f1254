"""API errors (``k8s.io/apimachinery/pkg/api/errors`` analogue) with ``metav1.Status`` wire form."""

from __future__ import annotations

from typing import Optional


class ApiError(Exception):
    def __init__(self, code: int, reason: str, message: str, details: Optional[dict] = None):
        super().__init__(message)
        self.code = code
        self.reason = reason
        self.message = message
        self.details = details or {}

    def to_status(self) -> dict:
        return {"kind": "Status", "apiVersion": "v1", "metadata": {}, "status": "Failure",
                "message": self.message, "reason": self.reason, "details": self.details, "code": self.code}

    @classmethod
    def from_status(cls, st: dict, http_code: int = 0) -> "ApiError":
        code = int(st.get("code") or http_code or 500)
        reason = st.get("reason") or _REASON_BY_CODE.get(code, "InternalError")
        cls_ = _CLASS_BY_REASON.get(reason, ApiError)
        err = cls_.__new__(cls_)
        ApiError.__init__(err, code, reason, st.get("message", ""), st.get("details"))
        return err

    def __repr__(self) -> str:
        return f"{type(self).__name__}({self.code} {self.reason}: {self.message})"


class NotFound(ApiError):
    def __init__(self, resource: str, name: str):
        super().__init__(404, "NotFound", f'{resource} "{name}" not found', {"name": name, "kind": resource})


class AlreadyExists(ApiError):
    def __init__(self, resource: str, name: str):
        super().__init__(409, "AlreadyExists", f'{resource} "{name}" already exists', {"name": name, "kind": resource})


class Conflict(ApiError):
    def __init__(self, resource: str, name: str, msg: str = ""):
        super().__init__(409, "Conflict",
                         f'Operation cannot be fulfilled on {resource} "{name}": '
                         f'{msg or "the object has been modified; please apply your changes to the latest version and try again"}',
                         {"name": name, "kind": resource})


class Invalid(ApiError):
    def __init__(self, resource: str, name: str, msg: str):
        super().__init__(422, "Invalid", f'{resource} "{name}" is invalid: {msg}', {"name": name, "kind": resource})


class BadRequest(ApiError):
    def __init__(self, msg: str):
        super().__init__(400, "BadRequest", msg)


class Forbidden(ApiError):
    def __init__(self, msg: str):
        super().__init__(403, "Forbidden", msg)


class NoKindMatch(ApiError):
    """``meta.IsNoMatchError``: the CRD for this kind is not installed."""

    def __init__(self, kind: str):
        super().__init__(404, "NoKindMatch", f'no matches for kind "{kind}" in version')


class Gone(ApiError):
    def __init__(self, msg: str = "too old resource version"):
        super().__init__(410, "Expired", msg)


class InternalError(ApiError):
    def __init__(self, msg: str):
        super().__init__(500, "InternalError", msg)


_REASON_BY_CODE = {400: "BadRequest", 403: "Forbidden", 404: "NotFound", 409: "Conflict", 410: "Expired",
                   422: "Invalid", 500: "InternalError"}
_CLASS_BY_REASON = {"NotFound": NotFound, "AlreadyExists": AlreadyExists, "Conflict": Conflict,
                    "Invalid": Invalid, "BadRequest": BadRequest, "Forbidden": Forbidden,
                    "NoKindMatch": NoKindMatch, "Expired": Gone, "Gone": Gone, "InternalError": InternalError}


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "NotFound"


def is_already_exists(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "AlreadyExists"


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "Conflict"


def is_invalid(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "Invalid"


def is_no_match(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.reason == "NoKindMatch"


def ignore_not_found(e: Optional[BaseException]) -> Optional[BaseException]:
    return None if e is None or is_not_found(e) else e
