"""Structured logging (same JSON record shape as the reference).

A JSON line carries: timestamp (UTC ISO-8601), level, logger, message, and when
available trace_id / span_id (from :mod:`vgate.tracing`), request_id, the keys
of ``extra={"extra_data": {...}}`` flattened in, and the formatted exception.
"""
from __future__ import annotations

import json
import logging
import os
import sys
from datetime import datetime, timezone
from typing import Any


def _trace_ids() -> tuple[str, str]:
    try:
        from vgate import tracing
        return tracing.current_ids()
    except Exception:  # noqa: BLE001
        return "", ""


class JSONFormatter(logging.Formatter):
    def format(self, record: logging.LogRecord) -> str:
        out: dict[str, Any] = {
            "timestamp": datetime.now(timezone.utc).isoformat(),
            "level": record.levelname,
            "logger": record.name,
            "message": record.getMessage(),
        }
        tid, sid = _trace_ids()
        if tid:
            out["trace_id"] = tid
            out["span_id"] = sid
        rid = getattr(record, "request_id", None)
        if rid is not None:
            out["request_id"] = rid
        extra = getattr(record, "extra_data", None)
        if extra:
            out.update(extra)
        if record.exc_info:
            out["exception"] = self.formatException(record.exc_info)
        return json.dumps(out, default=str)


class ConsoleFormatter(logging.Formatter):
    COLORS = {"DEBUG": "\033[36m", "INFO": "\033[32m", "WARNING": "\033[33m", "ERROR": "\033[31m",
              "CRITICAL": "\033[35m"}
    RESET = "\033[0m"

    def format(self, record: logging.LogRecord) -> str:
        c = self.COLORS.get(record.levelname, "")
        ts = datetime.now().strftime("%Y-%m-%d %H:%M:%S")
        msg = f"{c}[{ts}] {record.levelname:8}{self.RESET} {record.name}: {record.getMessage()}"
        extra = getattr(record, "extra_data", None)
        if extra:
            msg += " | " + " | ".join(f"{k}={v}" for k, v in extra.items())
        tid, sid = _trace_ids()
        if tid:
            msg += f" | trace_id={tid} span_id={sid}"
        if record.exc_info:
            msg += "\n" + self.formatException(record.exc_info)
        return msg


def setup_logging(level: str = "INFO", json_format: bool = True, logger_name: str = "vgate") -> logging.Logger:
    """Configure the ``vgate`` logger tree on stdout (propagate=False, like the reference)."""
    logger = logging.getLogger(logger_name)
    lvl = getattr(logging, str(level).upper(), logging.INFO)
    logger.setLevel(lvl)
    logger.handlers.clear()
    h = logging.StreamHandler(sys.stdout)
    h.setLevel(lvl)
    h.setFormatter(JSONFormatter() if json_format else ConsoleFormatter())
    logger.addHandler(h)
    logger.propagate = False
    return logger


def get_logger(name: str) -> logging.Logger:
    return logging.getLogger(name)


class LogContext:
    """``with LogContext(log, request_id=..):`` adds fields to every record of ``log``."""

    def __init__(self, logger: logging.Logger, **fields):
        self.logger = logger
        self.fields = fields
        self._filter = None

    def __enter__(self):
        fields = self.fields

        class _F(logging.Filter):
            def filter(self, record):
                extra = dict(getattr(record, "extra_data", None) or {})
                extra.update(fields)
                record.extra_data = extra
                return True

        self._filter = _F()
        self.logger.addFilter(self._filter)
        return self

    def __exit__(self, *exc):
        self.logger.removeFilter(self._filter)
        return False


# legacy env defaults (reference logging_config.py:213-214)
DEFAULT_LEVEL = os.getenv("VGATE_LOG_LEVEL", "INFO")
DEFAULT_JSON = os.getenv("VGATE_LOG_JSON", "true").lower() == "true"
