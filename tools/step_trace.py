"""Replay one workload's batched call K times (graph mode, nothing else in the
process) for clean rocprofv3 kernel traces (development aid).

    python tools/step_trace.py [workload] [steps]
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "sweep48"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
X = torch.from_numpy(bench.make_workload(name)).to("cuda:0")
md = bench.WORKLOADS[name][1]
kw = bench.CALL_KW.get(name, {})
for _ in range(steps):
    _, info = pkg.ripser_batch(X, maxdim=md, return_time=True, **kw)
print(f"{name}: last device_ms {info['device_ms']:.4f}")
