"""Typed error hierarchy + exit codes.

Parity: reference `src/utils/errors.ts:7-151` (ExitCode enum, RoundtableError
subclasses, substring classification of backend failures). The MI355X engine adds
two failure kinds that the reference never sees because it never owns a device:
``oom`` (HBM exhausted while growing a knight's KV) and ``device`` (HIP error /
unhealthy GPU group). Both are still surfaced as :class:`AdapterError` so the
orchestrator skip-the-knight semantics stay identical.
"""
from __future__ import annotations

import enum
from typing import Optional


class ExitCode(enum.IntEnum):
    SUCCESS = 0
    CONFIG_ERROR = 1
    ADAPTER_ERROR = 2
    SESSION_ERROR = 3
    FILE_WRITE_ERROR = 4
    CONSENSUS_ERROR = 5
    VALIDATION_ERROR = 6
    UNKNOWN = 99


class RoundtableError(Exception):
    """Base class; carries an exit code and an optional user-facing hint."""

    exit_code: ExitCode = ExitCode.UNKNOWN

    def __init__(self, message: str, exit_code: Optional[ExitCode] = None, *,
                 hint: Optional[str] = None, cause: Optional[BaseException] = None):
        super().__init__(message)
        self.message = message
        if exit_code is not None:
            self.exit_code = exit_code
        self.hint = hint
        self.cause = cause

    @property
    def name(self) -> str:
        return type(self).__name__


class ConfigError(RoundtableError):
    exit_code = ExitCode.CONFIG_ERROR


class SessionError(RoundtableError):
    exit_code = ExitCode.SESSION_ERROR


class ConsensusError(RoundtableError):
    exit_code = ExitCode.CONSENSUS_ERROR


class ValidationError(RoundtableError):
    exit_code = ExitCode.VALIDATION_ERROR


class FileWriteError(RoundtableError):
    exit_code = ExitCode.FILE_WRITE_ERROR

    def __init__(self, file_path: str, message: str, **kw):
        super().__init__(message, **kw)
        self.file_path = file_path


ADAPTER_ERROR_KINDS = ("not_installed", "timeout", "auth", "api", "oom", "device", "unknown")


class AdapterError(RoundtableError):
    exit_code = ExitCode.ADAPTER_ERROR

    def __init__(self, adapter: str, message: str, *, kind: str = "unknown", **kw):
        super().__init__(message, **kw)
        self.adapter = adapter
        self.kind = kind if kind in ADAPTER_ERROR_KINDS else "unknown"


class EngineTimeout(AdapterError):
    """Raised by the engine watchdog when a turn exceeds its wall-clock/step budget."""

    def __init__(self, adapter: str, message: str, **kw):
        super().__init__(adapter, message, kind="timeout", **kw)


class DeviceFlagError(AdapterError):
    """A bounded device-side wait expired during a turn (K9 one-shot all-reduce or persistent
    decode kernel error flag): the kernel proceeded on stale data, so the turn is failed."""


_CLASSIFIERS = (
    # (kind, substrings, message template, hint)
    ("not_installed", ("enoent", "not found", "not recognized", "command not found", "no such model"),
     "{a} backend not found: {m}", "Is the model for {a} configured in adapter_config?"),
    ("timeout", ("timeout", "timed out", "etimedout"),
     "{a} timed out: {m}", "Try increasing timeout_per_turn_seconds in .roundtable/config.json"),
    ("oom", ("out of memory", "hipErrorOutOfMemory".lower(), "oom"),
     "{a} ran out of device memory: {m}", "Reduce max_new_tokens / context, or give {a} more GPUs (tp)."),
    ("device", ("hip error", "hiperror", "device-side", "gpu hang", "unhealthy"),
     "{a} device error: {m}", "The knight's GPU group was marked unhealthy; it is skipped."),
    ("auth", ("api key", "apikey", "unauthorized", "401", "403"),
     "{a} authentication failed: {m}", "Check your API key or subscription for {a}."),
    ("api", ("api error", "rate limit", "429", "too many requests", "500", "502", "503"),
     "{a} API error: {m}", "Wait a moment and try again, or check your {a} usage limits."),
)


def classify_error(error: BaseException | str, adapter: str) -> AdapterError:
    """Map an arbitrary failure to an :class:`AdapterError` (errors.ts:86-126)."""
    if isinstance(error, AdapterError):
        return error
    msg = str(error)
    lower = msg.lower()
    cause = error if isinstance(error, BaseException) else None
    for kind, needles, tmpl, hint in _CLASSIFIERS:
        if any(n in lower for n in needles):
            return AdapterError(adapter, tmpl.format(a=adapter, m=msg), kind=kind,
                                hint=hint.format(a=adapter), cause=cause)
    return AdapterError(adapter, f"{adapter} error: {msg}", kind="unknown", cause=cause)


def format_error(error: RoundtableError) -> str:
    out = f"\n❌ {error.name}: {error.message}"
    if error.hint:
        out += f"\n\U0001f4a1 Hint: {error.hint}"
    if error.cause is not None:
        out += f"\n\U0001f50d Caused by: {error.cause}"
    return out


def get_exit_code(error: BaseException) -> int:
    if isinstance(error, RoundtableError):
        return int(error.exit_code)
    return int(ExitCode.UNKNOWN)
