import sys, numpy as np, torch
sys.path.insert(0, '.')
from whisperx_amd import _lib
from oracle import oracle
g = (0.0, 0.016875, 0.0619375)
for y in ([0, 1, 1], [1, 1, 1], [0, 1, 0], [1, 0, 1, 1, 1], [0.9] * 70, [0.1, 0.9] + [0.9] * 130):
    y = np.array(y, np.float32)
    (rs, re), = _lib.binarize([y], [g], 0.5, 0.363, 30)
    print(len(y), list(zip(rs.tolist(), re.tolist())), oracle.binarize(y, *g, 0.5, 0.363, max_duration=30))
