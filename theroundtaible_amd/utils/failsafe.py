"""First-contact failure containment for multi-rank runs (bench.py).

The reference never hangs on a broken knight: it classifies the failure and moves on
(/root/reference/src/utils/errors.ts:86-126, /root/reference/src/orchestrator.ts:521-535). A
multi-rank run has a harder version of that problem: a rank that fails or stalls leaves its
peers waiting inside a collective until the process-group timeout, and a watchdog abort there
prints nothing. This module gives every rank a named *stage* and a guard thread:

* a rank whose stage raises writes ``fail.r<rank>.json`` (stage, error) into a run directory
  shared by the node's ranks and exits non-zero;
* a rank whose current stage outlives its time limit does the same (``stalled``);
* rank 0's guard polls that directory: the first failure it sees — its own or a peer's — is
  printed as ONE JSON line naming the failed stage and rank, and the process exits non-zero
  without waiting for the collective its peers may be stuck in.

Fault injection for tests: ``ROUNDTABLE_BENCH_FAULT="<rank>:<stage>:raise|stall|sleep<s>"`` (comma
separated) raises, blocks, or pauses for <s> seconds on entry to that stage on that rank only.

Stages are tracked per thread (engines capture from their own threads) and every transition is
logged with a timestamp on stderr while a guard runs (or ``ROUNDTABLE_STAGE_LOG=1``).
"""
from __future__ import annotations

import contextlib
import json
import os
import shutil
import sys
import tempfile
import threading
import time
from typing import Callable, Dict, Optional

_lock = threading.RLock()   # re-entrant: the SIGTERM handler reads the stage on the main thread
# stage stack per thread: engines capture from their own threads (orchestrator.execute_plan), so
# a process-global stage saved / restored by overlapping sub-stages could restore a stale value;
# each thread keeps its own stack and the guard checks every thread's innermost stage
_stacks: Dict[int, list] = {}
_main = threading.main_thread().ident
_t_start = time.monotonic()
_guard: Optional["RunGuard"] = None


class FaultInjected(Exception):
    """Raised by an injected ``raise`` fault (never caught by recovery paths)."""


def current_stage() -> str:
    """The calling thread's innermost stage (else the main thread's, else ``start``)."""
    with _lock:
        st = _stacks.get(threading.get_ident()) or _stacks.get(_main)
        return st[-1][0] if st else "start"


def active_stages() -> list:
    """(name, entered at, own limit or None) of every thread's innermost stage."""
    with _lock:
        return [st[-1] for st in _stacks.values() if st]


def _log(name: str) -> None:
    if _guard is not None or os.environ.get("ROUNDTABLE_STAGE_LOG") == "1":
        # timestamped stage transitions on stderr: a run the launcher (or a silence watchdog)
        # kills still names the stage it was in
        rank = os.environ.get("RANK", "0")
        sys.stderr.write(f"[rank {rank} +{time.monotonic() - _t_start:8.2f}s] stage {name!r}\n")
        sys.stderr.flush()


def set_stage(name: str) -> str:
    """Enter stage ``name`` on the calling thread (replacing its innermost stage; returns the
    previous one); applies injected faults for it."""
    tid = threading.get_ident()
    with _lock:
        st = _stacks.setdefault(tid, [])
        prev = st[-1][0] if st else "start"
        if st:
            st[-1] = (name, time.monotonic(), None)
        else:
            st.append((name, time.monotonic(), None))
    _log(name)
    _maybe_fault(name)
    return prev


@contextlib.contextmanager
def stage(name: str, limit_s: Optional[float] = None):
    """A sub-stage (e.g. ``capture`` inside ``round 1``) of the calling thread: its enclosing
    stage resumes after it, with its own clock as it was. ``limit_s``: this stage's own time limit
    (else the guard's limit for its name)."""
    tid = threading.get_ident()
    with _lock:
        _stacks.setdefault(tid, []).append((name, time.monotonic(), limit_s))
    _log(name)
    try:
        _maybe_fault(name)
        yield
    finally:
        with _lock:
            st = _stacks.get(tid)
            if st:
                st.pop()
            if not st and tid != _main:
                _stacks.pop(tid, None)


def _maybe_fault(name: str) -> None:
    spec = os.environ.get("ROUNDTABLE_BENCH_FAULT", "")
    if not spec:
        return
    rank = int(os.environ.get("RANK", "0"))
    for item in spec.split(","):
        parts = item.split(":")
        if len(parts) != 3 or int(parts[0]) != rank or parts[1] != name:
            continue
        if parts[2] == "raise":
            raise FaultInjected(f"injected failure at stage {name!r} on rank {rank}")
        if parts[2] == "stall":
            while True:            # a stuck rank: only the guard (or the launcher) ends it
                time.sleep(1.0)
        if parts[2].startswith("sleep"):   # a rank that stalls for a while, then carries on
            time.sleep(float(parts[2][5:]))


def describe(rec: dict, prog: str) -> str:
    """One human line for a guard record (the CLI commands' report): the primary failure, then
    every other rank's record (a stall usually shows on several ranks at once: the stuck one and
    the ones waiting for it in a collective)."""
    line = f"{prog}: rank {rec.get('failed_rank')} failed at stage {rec.get('failed_stage')!r}: {rec.get('error')}"
    others = [r for r in rec.get("failures", []) if r.get("failed_rank") != rec.get("failed_rank")]
    if others:
        line += "; also " + "; ".join(
            f"rank {r.get('failed_rank')} {'stalled' if str(r.get('error', '')).startswith('stalled') else 'failed'} "
            f"at stage {r.get('failed_stage')!r}" for r in others)
    return line


def run_dir() -> str:
    """One directory per launch, shared by the ranks of this node: every rank of a torchrun
    launch has the same parent (the elastic agent) and master port."""
    key = f"{os.getppid()}-{os.environ.get('MASTER_PORT', '0')}" if "WORLD_SIZE" in os.environ else str(os.getpid())
    return os.path.join(tempfile.gettempdir(), f"rt-run-{key}")


class RunGuard:
    """Per-rank guard thread. ``limits``: stage-name prefix -> seconds (longest match wins),
    ``default_s`` otherwise. ``report(payload)`` prints rank 0's JSON line (called once)."""

    def __init__(self, rank: int, world: int, report: Callable[[dict], None], default_s: float = 300.0,
                 limits: Optional[Dict[str, float]] = None, poll_s: float = 0.25, ack_wait_s: float = 15.0,
                 exit_code: int = 3):
        self.rank, self.world, self.report = rank, world, report
        self.exit_code = exit_code
        self.ack_wait_s = ack_wait_s
        self.default_s, self.limits, self.poll_s = default_s, dict(limits or {}), poll_s
        self.dir = run_dir()
        self._done = False
        self._reported = False
        self._rlock = threading.Lock()
        os.makedirs(self.dir, exist_ok=True)    # (the key is per launch: no stale files to clear)

    def limit_for(self, name: str) -> float:
        best, n = self.default_s, -1
        for k, v in self.limits.items():
            if name.startswith(k) and len(k) > n:
                best, n = v, len(k)
        return best

    def start(self) -> "RunGuard":
        global _guard
        _guard = self
        if self.rank == 0 and self.world > 1 and threading.current_thread() is threading.main_thread():
            import signal
            signal.signal(signal.SIGTERM, self._on_term)
        threading.Thread(target=self._loop, name="roundtable-guard", daemon=True).start()
        return self

    def _loop(self) -> None:
        while not self._done:
            time.sleep(self.poll_s)
            now = time.monotonic()
            # every thread's innermost stage against its own limit; the most overdue one is named
            over = []
            for name, t0, own in active_stages():
                lim = own if own is not None else self.limit_for(name)
                if now - t0 > lim:
                    over.append((now - t0 - lim, name, lim))
            if over:
                _, name, lim = max(over)
                self.fail(name, f"stalled: stage {name!r} exceeded {lim:.0f} s on rank {self.rank}")
            if self.rank == 0:
                peer = self._peer_failure()
                if peer is not None:
                    self._report_and_exit(peer)

    def _records(self) -> list:
        try:
            files = sorted(f for f in os.listdir(self.dir) if f.startswith("fail."))
        except OSError:
            return []
        out = []
        for f in files:
            try:
                with open(os.path.join(self.dir, f)) as fh:
                    out.append(json.load(fh))
            except (OSError, ValueError):
                continue                         # being written: next poll
        return out

    def _peer_failure(self) -> Optional[dict]:
        recs = self._records()
        return recs[0] if recs else None

    def fail(self, stage_name: str, error: str) -> None:
        """Record this rank's failure and end the process (rank 0 reports it first)."""
        rec = {"failed_stage": stage_name, "failed_rank": self.rank, "error": error[:2000]}
        tmp = os.path.join(self.dir, f".fail.r{self.rank}.tmp")
        try:
            with open(tmp, "w") as fh:
                json.dump(rec, fh)
            os.replace(tmp, os.path.join(self.dir, f"fail.r{self.rank}.json"))
        except OSError:
            pass
        if self.rank == 0:
            self._report_and_exit(rec)
        sys.stderr.write(f"[rank {self.rank}] failed at stage {stage_name!r}: {error}\n")
        sys.stderr.flush()
        # the launcher tears every rank down as soon as one exits non-zero: stay until rank 0 has
        # printed the failure line (its ack file), bounded
        deadline = time.monotonic() + self.ack_wait_s
        while time.monotonic() < deadline and not os.path.exists(os.path.join(self.dir, "reported")):
            time.sleep(0.05)
        os._exit(self.exit_code)

    def _report_and_exit(self, rec: dict) -> None:
        with self._rlock:
            if not self._reported:
                self._reported = True
                # a stalled collective times out on every rank at about the same moment: give the
                # peers a moment to file theirs, then name a rank that RAISED if there is one (the
                # cause), else the first stalled record; every record rides along
                time.sleep(min(2.0, 8 * self.poll_s))
                recs = self._records() or [rec]
                raised = [r for r in recs if not str(r.get("error", "")).startswith("stalled")]
                primary = dict((raised or recs)[0])
                primary["failures"] = recs
                try:
                    self.report(primary)
                finally:
                    sys.stdout.flush()
                    sys.stderr.flush()
                    try:
                        open(os.path.join(self.dir, "reported"), "w").close()
                    except OSError:
                        pass
        os._exit(self.exit_code)

    def _on_term(self, signum, frame) -> None:  # noqa: ARG002 - signal handler signature
        """The launcher is tearing the run down (a peer exited): report what the peers filed."""
        recs = self._records()
        self._report_and_exit(recs[0] if recs else
                              {"failed_stage": current_stage(), "failed_rank": None,
                               "error": f"terminated by the launcher (signal {signum}) during stage "
                                        f"{current_stage()!r}"})

    def finish(self) -> None:
        """Normal end: stop the guard (rank 0 removes the run directory)."""
        self._done = True
        if self.rank == 0:
            shutil.rmtree(self.dir, ignore_errors=True)


def guard() -> Optional[RunGuard]:
    return _guard
