"""A/B of torch's BLAS backend for the emission forward (development tool):
python tools/blas_ab.py cublas|cublaslt  -> runs tools/legs.py e2e with that preferred library."""
import runpy
import sys

import torch

torch.backends.cuda.preferred_blas_library(sys.argv[1])
sys.argv = ["legs.py", "e2e", "--steps", "5", "--warmup", "2"]
runpy.run_path(__file__.replace("blas_ab.py", "legs.py"), run_name="__main__")
