"""Drop-in for src/clustering/clustering.py (same CLI flags).

    python clustering/clustering.py -i IN/ -o OUT/ -d track_state_estimates -c 1.0 -k 2.0 -l LUT -t 1 -z 0.4 -m 0.6 -b 550

cluster() loads the subgraphs (glob order), runs pairwise Mahalanobis chi2,
greedy merging with the KL distance, deferred in-edge deactivation, degree,
mixture weights and priors on the device (one fused node kernel,
clustering.py:181-373) and saves them renumbered. The LUT argument is accepted
and, as in the reference, unused (:149). ``-r`` (reset_reactivate, :126-146) is
broken in the reference (missing arguments) and raises here too.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gtf import stages as _st  # noqa: E402
from gtf.dropin import run_dir  # noqa: E402
from gtf.params import Params  # noqa: E402


def cluster(inputDir, outputDir, track_state_key, chi2_threshold, KL_threshold, KL_lut, iteration_num, reactivate,
            sigma0rz, sigma0rz2, endcap_boundary):
    if reactivate:
        raise TypeError("compute_track_state_estimates() missing 4 required positional arguments "
                        "(reference clustering.py:141)")
    p = Params(sigma0rz=sigma0rz, sigma0rz2=sigma0rz2, endcap_boundary=endcap_boundary)
    k = _st._key(track_state_key)
    # read -> one device call -> save, the pickle work on worker processes (gtf.dropin)
    run_dir(inputDir, outputDir, lambda d: d.cluster(k, chi2_threshold, KL_threshold, p))


def main():
    parser = argparse.ArgumentParser(description='edge outlier removal')
    parser.add_argument('-i', '--input', help='input directory of outlier removal')
    parser.add_argument('-o', '--output', help='output directory to save remaining network & track candidates')
    parser.add_argument('-d', '--dict', help='dictionary of track state estimates to use')
    parser.add_argument('-l', '--lut', help='lut file for KL distance acceptance region')
    parser.add_argument('-c', '--chi2', help='chi2 distance threshold')
    parser.add_argument('-k', '--kl', help='kl distance threshold')
    parser.add_argument('-t', '--iteration', help="iteration number")
    parser.add_argument('-r', '--reactivateall', default=False, type=bool)
    parser.add_argument('-z', '--sigma0rz', help="rms measurement error in rz plane")
    parser.add_argument('-m', '--sigma0rz2', help="rms measurement error in rz plane - Moliere MS orientation of layer is important")
    parser.add_argument('-b', '--endcapboundary', help="endcap boundary z coordinate - orientation of barrel and endcap layer")
    args = parser.parse_args()
    cluster(args.input, args.output, args.dict, float(args.chi2), float(args.kl), args.lut, int(args.iteration),
            args.reactivateall, float(args.sigma0rz), float(args.sigma0rz2), float(args.endcapboundary))


if __name__ == "__main__":
    main()
