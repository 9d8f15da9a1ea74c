"""Time the config-5 parabolic-KL section alone (diagnostics):

    python tools/pkl_time.py [steps] [--hot] [--f32]

Default: the cold rotation over 8 resident 256-event batches only (bench.bench_c5), fp64
only, so a profiler's per-kernel summary holds the roofline launches alone."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-track-finding_amd")]

import bench  # noqa: E402

if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    steps = int(args[0]) if args else 48
    dts = ("f64", "f32") if "--f32" in sys.argv else ("f64",)
    r = bench.bench_c5("cuda:0", steps, 2, hot="--hot" in sys.argv, dtypes=dts)
    print(json.dumps({"lib": os.environ.get("GTF_LIB", "default"),
                      **{dt + "_ms": r[dt]["kernel_ms"] for dt in dts},
                      **{dt + "_frac": r[dt]["roofline"]["frac"] for dt in dts},
                      "footprint": r["f64"]["roofline"]["footprint_bytes_all_batches"], "layout": r["layout"]}))
