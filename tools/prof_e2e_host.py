"""Development tool: cProfile of one warm align() call on the bench's e2e inputs (host-side time by function)."""
import cProfile, pstats, sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import bench, whisperx_amd
dev = torch.device("cuda", 0)
segs, audio, model, meta = bench.e2e_leg_inputs(dev)
for _ in range(2):
    whisperx_amd.align(segs, model, meta, audio, dev)
torch.cuda.synchronize()
t = time.perf_counter()
whisperx_amd.align(segs, model, meta, audio, dev)
torch.cuda.synchronize()
print("wall ms", (time.perf_counter() - t) * 1e3)
pr = cProfile.Profile()
pr.enable()
whisperx_amd.align(segs, model, meta, audio, dev)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
