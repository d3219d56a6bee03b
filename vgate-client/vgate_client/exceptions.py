"""SDK exception hierarchy: every error is a VGateError carrying the HTTP status and body."""
from __future__ import annotations

from typing import Any, Optional


class VGateError(Exception):
    def __init__(self, message: str, status_code: Optional[int] = None, body: Any = None):
        super().__init__(message)
        self.message = message
        self.status_code = status_code
        self.body = body

    def __str__(self) -> str:
        return f"[{self.status_code}] {self.message}" if self.status_code is not None else self.message


class AuthenticationError(VGateError):
    """401: missing or unknown API key."""


class RateLimitError(VGateError):
    """429: per-key sliding window exhausted. ``retry_after`` seconds from the server."""

    def __init__(self, message: str, retry_after: Optional[float] = None, status_code: Optional[int] = 429,
                 body: Any = None):
        super().__init__(message, status_code=status_code, body=body)
        self.retry_after = retry_after


class ServerError(VGateError):
    """5xx, a mid-stream error event, or a stream that ended without [DONE]."""


class ConnectionError(VGateError):  # noqa: A001 - public SDK name
    """The server could not be reached at all."""
