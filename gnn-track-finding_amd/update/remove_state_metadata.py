"""Drop-in for src/update/remove_state_metadata.py (same CLI flag -r).

Prunes state entries whose sender is no longer a successor of the node, then
recomputes priors on both state dicts and reweights (remove_state_metadata.py:
29-53) in one device call; saves the graphs back renumbered in glob order.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from gtf.dropin import run_dir  # noqa: E402
from gtf.params import Params  # noqa: E402


def main():
    parser = argparse.ArgumentParser(description='extract track candidates')
    parser.add_argument('-r', '--remain', help='output directory to save remaining network')
    args = parser.parse_args()
    # read -> one device call -> save in place, the pickle work on worker processes
    # (gtf.dropin; every file is read before any is written)
    p = Params()
    run_dir(args.remain, args.remain, lambda d: d.update(p))


if __name__ == "__main__":
    main()
