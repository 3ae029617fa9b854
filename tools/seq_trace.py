"""One sweep48 call at a time (graph replay, the bench's `sequential` figure),
for a rocprofv3 kernel trace read by tools/timeline.py (dev aid):
    rocprofv3 --kernel-trace -d gpurun_out/seq -- python tools/seq_trace.py [L] [calls] [one_stream 0|1]"""
import importlib
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
L = int(sys.argv[1]) if len(sys.argv) > 1 else 32
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 30
kw = {"input_ready": True}
if len(sys.argv) > 3:
    kw["one_stream"] = sys.argv[3] == "1"
X = torch.from_numpy(bench.make_workload("sweep48", L)).to("cuda:0")
torch.cuda.synchronize()
for _ in range(5):
    pkg.ripser_batch(X, maxdim=2, **kw)
torch.cuda.synchronize()
dev = []
t0 = time.perf_counter()
for _ in range(calls):
    _, info = pkg.ripser_batch(X, maxdim=2, return_time=True, **kw)
    dev.append(info["device_ms"])
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / calls * 1e3
dev.sort()
print(f"L={L} {kw}: wall {wall:.4f} ms/call, device median {dev[len(dev) // 2]:.4f} ms (min {dev[0]:.4f})", flush=True)
