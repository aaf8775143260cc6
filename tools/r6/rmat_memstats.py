"""bench.py --workload rmat with the caching allocator's counters printed at exit (diagnostic:
allocation retries free cached blocks, which synchronises the device)."""
import atexit
import os
import runpy
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))


def report():
    st = torch.cuda.memory_stats()
    keys = ("num_alloc_retries", "num_ooms", "num_device_alloc", "num_device_free", "num_sync_all_streams",
            "allocated_bytes.all.peak", "reserved_bytes.all.peak")
    print("memstats", {k: st.get(k) for k in keys}, file=sys.stderr, flush=True)


atexit.register(report)
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "bench.py"), run_name="__main__")
