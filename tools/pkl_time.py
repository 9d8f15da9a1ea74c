"""Time the config-5 parabolic-KL section alone (diagnostics): python tools/pkl_time.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-track-finding_amd")]

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    r = bench.bench_c5("cuda:0", steps, 5)
    print(json.dumps({"lib": os.environ.get("GTF_LIB", "default"), "f64_ms": r["f64"]["kernel_ms"],
                      "f32_ms": r["f32"]["kernel_ms"], "f64_frac": r["f64"]["roofline"]["frac"],
                      "f32_frac": r["f32"]["roofline"]["frac"], "sweep": r["fp32_vs_fp64"]}))
