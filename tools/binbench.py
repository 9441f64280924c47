"""Binarize / merge_chunks timing on 1 h of synthetic VAD scores (development tool; library
from WX_LIB_PATH when set, for A/B)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from whisperx_amd import synthetic  # noqa: E402
from whisperx_amd.vad import merge_chunks  # noqa: E402

sc = synthetic.vad_scores(3, 3600.0)
merge_chunks(sc, 30, 0.5, 0.363)
torch.cuda.synchronize()
ts = []
for _ in range(10):
    t0 = time.perf_counter()
    ch = merge_chunks(sc, 30, 0.5, 0.363)
    ts.append(time.perf_counter() - t0)
print(f"{os.environ.get('WX_LIB_PATH', 'in-tree')}: merge_chunks 1 h min {1000 * min(ts):.2f} ms, "
      f"median {1000 * sorted(ts)[5]:.2f} ms, {len(ch)} chunks", flush=True)
