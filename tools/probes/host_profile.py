"""Host-side profile of a bench run: cProfile with every ThreadPoolExecutor task run inline on the
main thread (cProfile sees only the thread it runs on; the orchestrator runs each engine group
on a pool thread). Arguments after the script are bench.py's.

    python tools/probes/host_profile.py --out gpurun_out/prof.txt -- --simulate-tp 8 --steps 3 --warmup 1
"""
from __future__ import annotations

import concurrent.futures as cf
import cProfile
import io
import os
import pstats
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _Inline(cf.Executor):
    def __init__(self, *a, **k):
        pass

    def submit(self, fn, *args, **kwargs):
        f = cf.Future()
        try:
            f.set_result(fn(*args, **kwargs))
        except BaseException as e:  # noqa: BLE001 - handed to the caller like a pool would
            f.set_exception(e)
        return f

    def shutdown(self, wait=True, **kw):
        pass


def main() -> int:
    argv = sys.argv[1:]
    out = "host_profile.txt"
    if "--out" in argv:
        i = argv.index("--out")
        out = argv[i + 1]
        del argv[i:i + 2]
    if argv and argv[0] == "--":
        argv = argv[1:]
    cf.ThreadPoolExecutor = _Inline
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv
    sys.path.insert(0, ROOT)
    prof = cProfile.Profile()
    prof.enable()
    try:
        runpy.run_path(sys.argv[0], run_name="__main__")
    except SystemExit:
        pass
    prof.disable()
    s = io.StringIO()
    st = pstats.Stats(prof, stream=s)
    st.sort_stats("cumulative").print_stats(r"theroundtaible_amd|bench", 80)
    st.sort_stats("tottime").print_stats(40)
    with open(out, "w") as f:
        f.write(s.getvalue())
    return 0


if __name__ == "__main__":
    sys.exit(main())
