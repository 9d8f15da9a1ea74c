"""Stage parameters with the reference's defaults.

The reference passes these as argparse flags from run_gnn_trackml_mod.sh:7-37
(sigma0xy 0.3, sigma0rz 0.4, sigma0rz2 0.6, endcap 550, extrapolation chi2 cut
2.0) and hard-codes the reweight threshold (helper.py:145). The clustering
thresholds are per iteration: -c 1.0 -k 2.0 on track_state_estimates
(run_gnn_trackml_mod.sh:89), -c 1000 -k 100 on updated_track_states (:112).
"""
import dataclasses


@dataclasses.dataclass
class Params:
    sigma0xy: float = 0.3
    sigma0rz: float = 0.4
    sigma0rz2: float = 0.6
    endcap_boundary: float = 550.0
    chi2_cut: float = 2.0            # extrapolation gate, extrapolate_merged_states.py:298
    reweight_threshold: float = 0.1  # helper.py:145
    cluster_chi2: float = 1000.0     # clustering.py:228 (iteration >= 3 value)
    cluster_kl: float = 100.0        # clustering.py:261
    tag_threshold: float = 0.1       # tag_propagation.py:130
