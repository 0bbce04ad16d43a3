"""gfp_gaussian_process_amd -- MI355X-native lineage-tree likelihood for gfp_gaussian_process.

The hot path (per-cell Kalman update + closed-form OU/Dawson propagator + division map,
summed over a lineage forest) runs as FP64 HIP kernels for gfx950 in lib/libggp.so,
behind the C-ABI of include/ggp.h.  This package is the thin host-side mirror of the
reference's objective entry points (see forest.py for the mapping).
"""
from .forest import (  # noqa: F401
    CSVConfig, Dataset, EvaluationStalled, Forest, GGPError, HostForest, LikelihoodIsNan, ParameterSet,
    PARAM_NAMES, total_likelihood, total_likelihood_log_params, total_likelihood_nlopt,
)

__all__ = [
    "CSVConfig", "Dataset", "EvaluationStalled", "Forest", "GGPError", "HostForest", "LikelihoodIsNan", "ParameterSet",
    "PARAM_NAMES", "total_likelihood", "total_likelihood_log_params", "total_likelihood_nlopt",
]
