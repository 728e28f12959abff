"""GPU diagnostics on the sample stream -- drop-ins
for the reference's ``src/diagnostics/mcmc_diag.py`` and
``src/diagnostics/convergence_diag.py`` plus the sampler-base moments
(``src/samplers/base.py:154-160``).  Kernels: ``csrc/lgs_diag.hip``."""
from . import convergence_diag, mcmc_diag, moments  # noqa: F401
from .convergence_diag import (batch_means_variance, compute_ess_per_second, compute_tvd,  # noqa: F401
                               gelman_rubin_statistic, mixing_time_estimate, spectral_gap_estimate)
from .mcmc_diag import (compute_acceptance_rate, compute_autocorrelation, compute_jump_distance,  # noqa: F401
                        compute_mcse, diagnose_chain, effective_sample_size,
                        integrated_autocorrelation_time)
from .moments import empirical_covariance, empirical_mean, empirical_std, gram  # noqa: F401
