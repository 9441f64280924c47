"""End-to-end probe (development tool, GPU box): bench.py's config-3 leg (1 h -> VAD -> ~120
chunks -> align()) with align()'s phase times (WX_PROFILE=1), MIOpen convolutions vs the GEMM
route, and the fixed-length e2e leg."""
import json
import os
import sys

os.environ["WX_PROFILE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from whisperx_amd import alignment  # noqa: E402


def run(label, fn):
    alignment.PHASE_TIMES.clear()
    r = fn()
    r["phases_ms"] = {k: round(1000 * v, 1) for k, v in alignment.PHASE_TIMES.items()}
    print(label, json.dumps(r), flush=True)


def main():
    dev = torch.device("cuda", 0)
    variants = sys.argv[1:] or ["miopen", "gemm"]
    for v in variants:
        if v == "miopen":
            os.environ["WX_MIOPEN_CONV"] = "1"
        else:
            os.environ.pop("WX_MIOPEN_CONV", None)
        run(f"config3[{v}]", lambda: bench.e2e_config3(dev))
        run(f"e2e30[{v}]", lambda: bench.e2e_align(dev))


if __name__ == "__main__":
    main()
