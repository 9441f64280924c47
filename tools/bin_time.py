#!/usr/bin/env python
"""Development tool: bench.py's binarize_1h leg alone (for rocprofv3 kernel stats)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

print(json.dumps(bench.binarize_1h("cuda:0")), flush=True)
