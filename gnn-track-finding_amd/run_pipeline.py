"""run_gnn_trackml_mod.sh (:7-146) as one process: event conversion and iterations
START..END of clustering / extrapolation -> candidate extraction -> metadata update,
every stage on the GPU (gtf.pipeline), stage outputs saved in the compact packed
format (gtf.store) instead of per-subgraph gpickles.

    python run_pipeline.py -n <event_network dir> -o <ROOTDIR> -a 7 -z 7 [--start 1 --end 3]

Layout under ROOTDIR (the run script's directories, one file each):

    track_sim/network/graph.npz              event conversion output
    iteration_i/network/graph.npz            the iteration's stage output
    iteration_i/candidates/candidates.npz    extracted candidates (node ids) + p-values
    iteration_i/candidates/pvals.csv         as extract_track_candidates.py writes it (:485-486)
    iteration_i/remaining/graph.npz          the next iteration's input (after update on even i)
    iteration_i/fragments/fragments.npz      node ids of the track fragments
    timings.json                             wall time per stage
    metrics.json                             with --truth: reconstruction efficiency and purities
                                             (gtf.metrics; the run script's last step, :143-146)

--start S > 1 resumes from ROOTDIR/iteration_{S-1}/remaining/graph.npz, as the run
script's commented "iteration by iteration" mode does (:79-81).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)

from gtf import extract, pipeline, store  # noqa: E402
from gtf.params import Params  # noqa: E402


def _dir(*parts):
    d = os.path.join(*parts)
    os.makedirs(d, exist_ok=True)
    return d


def main(argv=None):
    ap = argparse.ArgumentParser(description="GNN track finding on the GPU (run_gnn_trackml_mod.sh)")
    ap.add_argument("-n", "--eventNetwork", help="directory holding event_1_filtered_graph_{nodes,edges}.csv")
    ap.add_argument("-o", "--outputDir", required=True, help="ROOTDIR")
    ap.add_argument("-a", "--min_volume", type=int, default=7)
    ap.add_argument("-z", "--max_volume", type=int, default=7)
    ap.add_argument("-e", "--sigma0xy", type=float, default=0.3)
    ap.add_argument("-r", "--sigma0rz", type=float, default=0.4)
    ap.add_argument("-m", "--sigma0rz2", type=float, default=0.6)
    ap.add_argument("-b", "--endcapboundary", type=float, default=550.0)
    ap.add_argument("-c", "--chi2", type=float, default=2.0, help="extrapolation chi2 cut (c)")
    ap.add_argument("-p", "--pval", type=float, default=0.01)
    ap.add_argument("--numhits", type=int, default=4, help="n")
    ap.add_argument("-s", "--separation", type=float, default=10.0)
    ap.add_argument("-t", "--merge", type=float, default=8.0, help="threshold distance node merging")
    ap.add_argument("--start", type=int, default=1)
    ap.add_argument("--end", type=int, default=3)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--truth", help="EVENT_TRUTH dir: score the candidates (reconstruction_efficiency.py)")
    ap.add_argument("--mapping", default="full-mapping-minCurv-0.3-800.csv", help="mapping file under --truth")
    args = ap.parse_args(argv)
    if args.start < 1 or args.end < args.start:
        ap.error("need 1 <= start <= end")
    p = Params(sigma0xy=args.sigma0xy, sigma0rz=args.sigma0rz, sigma0rz2=args.sigma0rz2,
               endcap_boundary=args.endcapboundary, chi2_cut=args.chi2)
    ex = extract.Params(args.pval, args.numhits, args.separation, args.merge, args.sigma0xy, args.sigma0rz,
                        args.endcapboundary)
    root = args.outputDir
    times = {}
    if args.start == 1:
        if not args.eventNetwork:
            ap.error("-n is required when starting at iteration 1")
        t0 = time.perf_counter()
        g, vivl = pipeline.build_event(os.path.join(args.eventNetwork, "event_1_filtered_graph_"), args.min_volume,
                                       args.max_volume, p, args.device)
        times["event_conversion"] = time.perf_counter() - t0
        store.save_graph(os.path.join(_dir(root, "track_sim", "network"), "graph.npz"), g, vivl)
        print("event conversion: %d nodes, %d directed edges, %d subgraphs (%.3f s)"
              % (g.n_nodes, g.n_edges, g.n_subgraphs, times["event_conversion"]))
    else:
        g, vivl = store.load_graph(os.path.join(root, "iteration_%d" % (args.start - 1), "remaining", "graph.npz"))
        if vivl is None:
            raise SystemExit("remaining graph has no vivl array")
    its = pipeline.run(g, vivl, args.end - args.start + 1, p, ex, args.device, first=args.start, keep_graphs=True)
    for it in its:
        d = os.path.join(root, "iteration_%d" % it.index)
        store.save_graph(os.path.join(_dir(d, "network"), "graph.npz"), it.network)
        cdir = _dir(d, "candidates")
        store.save_groups(os.path.join(cdir, "candidates.npz"), it.candidates, pval_xy=it.pval_xy,
                          pval_zr=it.pval_zr)
        with open(os.path.join(cdir, "pvals.csv"), "w") as f:
            f.write(",pvals_xy,pvals_zr\n")
            for i, (a, b) in enumerate(zip(it.pval_xy, it.pval_zr)):
                f.write("%d,%r,%r\n" % (i, float(a), float(b)))
        store.save_graph(os.path.join(_dir(d, "remaining"), "graph.npz"), it.remaining_graph, it.remaining_vivl)
        store.save_groups(os.path.join(_dir(d, "fragments"), "fragments.npz"), it.fragments)
        times["iteration_%d" % it.index] = it.seconds
        print("iteration %d (%s): %d candidates, %d remaining, %d fragments"
              % (it.index, it.stage, len(it.candidates), len(it.remaining), len(it.fragments)))
    with open(os.path.join(_dir(root), "timings.json"), "w") as f:
        json.dump(times, f, indent=1)
    if args.truth and its:
        from extract import reconstruction_efficiency as re_cli
        from gtf import metrics
        res = {}
        for name, cum in (("last_iteration", False), ("cumulative", True)):
            r = re_cli.score(args.truth, root, args.min_volume, args.max_volume, its[-1].index, args.mapping, cum)
            res[name] = metrics.summary(r)
            print("%s: %d / %d reference tracks reconstructed, efficiency %s %%"
                  % (name, r.n_reconstructed, r.n_reference, r.efficiency_str))
        with open(os.path.join(root, "metrics.json"), "w") as f:
            json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
