"""Wall time of run_gnn_trackml_mod.sh's stages (START=1 END=3) with the drop-in CLIs,
each in its own process as the script runs them, on the committed vol-7 134 event
(truth mapping from tests/golden, as tests/test_pipeline.py's chain test):

    python tools/run_script_time.py OUT.json
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "gnn-track-finding_amd")
sys.path[:0] = [os.path.join(ROOT, "tests"), PKG, ROOT]


def main(path):
    from test_event_conversion import _truth_frame
    tmp = tempfile.mkdtemp()
    root, net, tru = tmp + "/output", tmp + "/net", tmp + "/truth"
    os.makedirs(net)
    os.makedirs(tru)
    kat = os.path.join(ROOT, "tests", "golden", "kat134", "event_1_filtered_graph_")
    for f in ("nodes.csv", "edges.csv"):
        with open(kat + f) as a, open(os.path.join(net, "event_1_filtered_graph_" + f), "w") as b:
            b.write(a.read())
    _truth_frame().to_csv(os.path.join(tru, "event000001000-full-mapping-minCurv-0.3-800.csv"), index=False)
    sz = ["-z", "0.4", "-m", "0.6", "-b", "550.0"]
    stages = []

    prof = os.environ.get("GTF_PROFILE_STAGE")   # e.g. it1_extract: cProfile that stage (top functions to stdout)

    def cli(name, module, *args):
        t = time.perf_counter()
        pre = ["-m", "cProfile", "-s", "cumulative"] if name == prof else []
        r = subprocess.run([sys.executable] + pre + [os.path.join(PKG, module)] + list(args), check=True,
                           env=dict(os.environ, GTF_REUSE_TRUTH_MAPPING="1"),
                           capture_output=True, text=True)
        if pre:
            print("\n".join(r.stdout.splitlines()[:60]))
        stages.append((name, time.perf_counter() - t))
        print(name, "%.3f s" % stages[-1][1], flush=True)

    inp = root + "/track_sim/network/"
    os.makedirs(inp)
    cli("event_conversion", "trackml_mod/event_conversion.py", "-o", inp, "-n", net, "-t", tru, "-a", "7", "-z", "7",
        "-e", "0.3", "-r", "0.4", "-m", "0.6", "-b", "550.0")
    for i in (1, 2, 3):
        out = root + "/iteration_%d/network/" % i
        os.makedirs(out)
        if i == 1:
            cli("it1_clustering", "clustering/clustering.py", "-i", inp, "-o", out, "-d", "track_state_estimates",
                "-c", "1.0", "-k", "2.0", "-l", "x.lut", "-t", "1", *sz)
        elif i % 2 == 0:
            cli("it%d_extrapolation" % i, "extrapolate/extrapolate_merged_states.py", "-i", inp, "-o", out, "-c", "2.0",
                "-e", "0.3", *sz)
        else:
            cli("it%d_clustering" % i, "clustering/clustering.py", "-i", inp, "-o", out, "-d", "updated_track_states",
                "-c", "1000", "-k", "100", "-l", "x.lut", "-t", str(i), *sz)
        cand, rem, frag = (root + "/iteration_%d/%s/" % (i, k) for k in ("candidates", "remaining", "fragments"))
        for d in (cand, rem, frag):
            os.makedirs(d)
        if i > 1:
            subprocess.check_call(["cp", "-r", root + "/iteration_%d/candidates/" % (i - 1), cand])
        cli("it%d_extract" % i, "extract/extract_track_candidates.py", "-i", out, "-c", cand, "-r", rem, "-f", frag,
            "-p", "0.01", "-n", "4", "-s", "10", "-t", "8.0", "-a", str(i), "-e", "0.3", "-z", "0.4", "-b", "550.0")
        if i % 2 == 0:
            cli("it%d_update" % i, "update/remove_state_metadata.py", "-r", rem)
        inp = rem
    res = {"stages_s": dict(stages), "total_s": sum(t for _, t in stages),
           "note": "run_gnn_trackml_mod.sh START=1 END=3 on the vol-7 134 event, every stage a drop-in CLI process"}
    print(json.dumps(res))
    with open(path, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])
