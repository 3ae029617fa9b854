"""Device-inclusive wall time of the reference's UMAP step for a 32-layer
sweep (36 prompts x 4096 features, n_neighbors 6, 3 components, cosine,
500 epochs) on the GPU (dev aid)."""
import importlib
import os
import statistics
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

pkg = importlib.import_module("tda-multimodal_amd")
X = torch.from_numpy(pkg.synthetic.activations(32, 36, 4096)).to("cuda:0")
kw = dict(n_neighbors=6, n_components=3, min_dist=0.1, metric="cosine", random_state=42)
pkg.umap_batch(X, **kw)
ts = []
for _ in range(10):
    t0 = time.perf_counter()
    Y = pkg.umap_batch(X, **kw)
    ts.append(time.perf_counter() - t0)
print(f"umap 32 x 36 x 4096: {statistics.median(ts) * 1e3:.2f} ms per sweep ({32 / statistics.median(ts):.0f} layers/s), "
      f"finite={bool(np.all(np.isfinite(Y)))}", flush=True)
