#!/usr/bin/env python3
"""Poor man's sampling profiler for the bench's host side: a daemon thread samples every
thread's Python stack every ~0.5 ms while bench.main() runs and prints inclusive / leaf
counts per function (threads included, unlike cProfile). Waits inside GPU synchronisation
show up as the frames that block (tolist, synchronize, replay).

Usage: python tools/host_sampler.py [bench args...] > out.txt
"""
import collections
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    incl = collections.Counter()
    leaf = collections.Counter()
    n = [0]
    stop = threading.Event()
    me = threading.get_ident()

    def sampler():
        while not stop.is_set():
            for tid, fr in sys._current_frames().items():
                if tid == me_sampler[0]:
                    continue
                seen = set()
                f = fr
                first = True
                while f is not None:
                    key = f"{os.path.basename(f.f_code.co_filename)}:{f.f_code.co_name}"
                    if first:
                        leaf[key] += 1
                        first = False
                    if key not in seen:
                        incl[key] += 1
                        seen.add(key)
                    f = f.f_back
            n[0] += 1
            time.sleep(0.0005)

    me_sampler = [None]
    th = threading.Thread(target=lambda: (me_sampler.__setitem__(0, threading.get_ident()), sampler()),
                          daemon=True)
    sys.argv = ["bench.py"] + sys.argv[1:]
    import bench
    th.start()
    try:
        bench.main()
    finally:
        stop.set()
        th.join()
    del me
    print(f"# samples {n[0]}")
    print("## inclusive (top 60)")
    for k, v in incl.most_common(60):
        print(f"{v:8d}  {k}")
    print("## leaf (top 40)")
    for k, v in leaf.most_common(40):
        print(f"{v:8d}  {k}")


if __name__ == "__main__":
    main()
