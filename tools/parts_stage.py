"""Stage times of one 128-layer call given as one array vs as 4 parts (dev aid)."""
import importlib
import os
import sys

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

torch.cuda.init()
pkg = importlib.import_module("tda-multimodal_amd")
X = pkg.synthetic.sweep48(32)
Xt = torch.from_numpy(X).cuda()
X4 = torch.from_numpy(np.concatenate([X] * 4)).cuda()
for tag, arg in (("one array", X4), ("4 parts", [Xt] * 4), ("one array", X4), ("4 parts", [Xt] * 4), ("32 layers", Xt)):
    for serial in (True, False):
        for _ in range(3):
            res, info = pkg.ripser_batch(arg, maxdim=2, return_time=True, stage_times=True, stage_serial=serial)
        st = dict(info["stages"])
        print(f"{tag:10s} serial={serial}: device {info['device_ms']:.4f} ms  chain {st.get('k_h1_chain', 0):.4f}  "
              f"phase1 {st.get('k_h2_phase1', 0):.4f}  app2 {st.get('k_apparent<2>', 0):.4f}  cs0 {res[0].checksum}", flush=True)
