"""Drop-in for src/extrapolate/extrapolate_merged_states.py (same CLI flags).

    python extrapolate/extrapolate_merged_states.py -i IN/ -o OUT/ -c 2.0 -e 0.3 -z 0.4 -m 0.6 -b 550

main() reads every ``*_subgraph.gpickle`` of the input directory (glob order,
:544-548), runs message passing + priors/reweight x2 + node degree as one fused
HIP call (gtf_extrapolate, :552-566) and saves the graphs renumbered in the
same order (:570-571); the pickle reading / writing runs on worker processes
(gtf.dropin.run_dir). The per-edge diagnostic CSVs and prints of the reference
(:143-295, :496-518) have no effect on outputs and are not produced.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gtf import stages as _st  # noqa: E402
from gtf.dropin import run_dir  # noqa: E402
from gtf.params import Params  # noqa: E402


def message_passing(subGraphs, chi2CutFactor, sigma0xy, sigma0rz, sigma0rz2, endcap_boundary):
    """:406-451 -- extrapolate every merged state along active out-edges"""
    _st.message_passing(subGraphs, chi2CutFactor, sigma0xy, sigma0rz, sigma0rz2, endcap_boundary)


def main():
    parser = argparse.ArgumentParser(description='edge outlier removal')
    parser.add_argument('-i', '--inputDir', help='input directory of outlier removal')
    parser.add_argument('-o', '--outputDir', help='output directory for updated states')
    parser.add_argument('-c', '--chi2CutFactor', help='chi2 cut factor for threshold')
    parser.add_argument('-e', '--sigma0xy', help="rms measurement error in xy")
    parser.add_argument('-z', '--sigma0rz', help="rms measurement error in rz")
    parser.add_argument('-m', '--sigma0rz2', help="rms measurement error in rz - MS Moliere orientation of layer important")
    parser.add_argument('-b', '--endcapboundary', help="endcap boundary z coordinate - orientation of barrel and endcap layer")
    args = parser.parse_args()
    p = Params(sigma0xy=float(args.sigma0xy), sigma0rz=float(args.sigma0rz), sigma0rz2=float(args.sigma0rz2),
               endcap_boundary=float(args.endcapboundary), chi2_cut=float(args.chi2CutFactor))
    # read -> one fused device call -> save, the per-file pickle work on worker processes
    # (gtf.dropin: same outputs and file numbering as the loop over read_subgraphs)
    run_dir(args.inputDir, args.outputDir, lambda d: d.extrapolate(p))


if __name__ == "__main__":
    main()
