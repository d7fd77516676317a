"""distributedlpsolver_amd — MI355X-native dense-tableau fp64 simplex.

The drop-in for the per-iteration solver core of shidanxu/DistributedLPSolver
(SURVEY.md §8).  Compute lives in libdlp.so (hand-written gfx950 HIP kernels
behind the C ABI of include/dlp.h); this package is the thin host binding.
"""
from ._lib import (NativeLibraryMissing, DLPError, OK, INFEASIBLE, UNBOUNDED, PIVOT_LIMIT,  # noqa: F401
                   RUNNING, PRICING_DANTZIG_BLAND, PRICING_BLAND, MINIMIZE, MAXIMIZE, lib)
from .solver import (Problem, Result, Session, BatchResult, solve, batched_solve, batched_occupancy, options,  # noqa: F401
                     rank_rows, candidate_select, tableau_ld, device_count, comm_unique_id, release_cached_memory,
                     PIVOT_DTYPE, CAND_DTYPE, MW, MW_ITER_DTYPE)

__all__ = ["Problem", "Result", "Session", "solve", "batched_solve", "batched_occupancy", "options", "rank_rows",
           "candidate_select", "tableau_ld", "device_count", "comm_unique_id", "release_cached_memory", "lib",
           "NativeLibraryMissing", "DLPError"]
