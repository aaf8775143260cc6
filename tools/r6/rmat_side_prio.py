"""bench.py --workload rmat with the side stream pre-created at a given priority (diagnostic A/B:
SIDE_PRIO=0 normal, -1 high)."""
import os
import runpy
import sys
import threading

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from spmm_amd.ops import spgemm as SG  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
SG._SIDE[(dev.index, threading.get_ident())] = torch.cuda.Stream(dev, priority=int(os.environ.get("SIDE_PRIO", "-1")))
sys.argv = ["bench.py"] + sys.argv[1:]
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "bench.py"), run_name="__main__")
