"""Crash-safe file primitives for the `.roundtable/` shared brain.

The reference rewrites ``status.json``/``manifest.json``/``decree-log.json``/
``chronicle.md`` in place with read-merge-write and no locking
(`src/utils/session.ts:120-149`, `src/utils/manifest.ts:41-52`,
`src/utils/decree-log.ts:66-70`, `src/utils/chronicle.ts:34-53`).
Here every write is temp-file + fsync + rename, and read-merge-write sequences run
under an advisory ``flock`` so two concurrent ``roundtable`` processes in one
project cannot tear each other's files.
"""
from __future__ import annotations

import contextlib
import fcntl
import os
import tempfile
from typing import Iterator


def atomic_write_text(path: str, text: str) -> None:
    d = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp-", dir=d)
    try:
        with os.fdopen(fd, "w", encoding="utf-8", newline="") as f:
            f.write(text)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        with contextlib.suppress(OSError):
            os.unlink(tmp)
        raise


def read_text(path: str) -> str:
    with open(path, "r", encoding="utf-8", newline="") as f:
        return f.read()


@contextlib.contextmanager
def file_lock(path: str) -> Iterator[None]:
    """Exclusive advisory lock on ``<path>.lock`` (created on demand)."""
    lock_path = path + ".lock"
    os.makedirs(os.path.dirname(os.path.abspath(lock_path)) or ".", exist_ok=True)
    fd = os.open(lock_path, os.O_RDWR | os.O_CREAT, 0o644)
    try:
        fcntl.flock(fd, fcntl.LOCK_EX)
        yield
    finally:
        with contextlib.suppress(OSError):
            fcntl.flock(fd, fcntl.LOCK_UN)
        os.close(fd)


class SessionLock:
    """PID lock on a session directory (TODO.md:188's stale-lock idea, implemented).

    A lock whose PID is no longer alive is considered stale and is taken over.
    """

    def __init__(self, session_path: str):
        self.path = os.path.join(session_path, ".lock")
        self.held = False

    def acquire(self) -> bool:
        for _ in range(2):
            try:
                fd = os.open(self.path, os.O_WRONLY | os.O_CREAT | os.O_EXCL, 0o644)
                with os.fdopen(fd, "w") as f:
                    f.write(str(os.getpid()))
                self.held = True
                return True
            except FileExistsError:
                try:
                    pid = int(read_text(self.path).strip() or "0")
                except (OSError, ValueError):
                    pid = 0
                if pid and _pid_alive(pid) and pid != os.getpid():
                    return False
                with contextlib.suppress(OSError):
                    os.unlink(self.path)
        return False

    def release(self) -> None:
        if self.held:
            with contextlib.suppress(OSError):
                os.unlink(self.path)
            self.held = False

    def __enter__(self):
        self.acquire()
        return self

    def __exit__(self, *exc):
        self.release()


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        return True
    return True
