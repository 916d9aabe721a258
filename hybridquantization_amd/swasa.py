"""Mirror of the reference's ``SWASA`` parameter object (SW:3-116).

The policy itself (RNG, neighbours, acceptance, temperature, convergence) runs
natively inside libhq (hq_swasa.h / hq_host.cpp) so the search loop has no
Python in it.  ``icy.util.Random`` is unseeded in the reference (SW:46); here
the generator is ``java.util.Random``-compatible and seeded explicitly.
"""

from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, load


class SWASA:
    """SW:14 ``SWASA(population, imax, iTc, delta, convDelay, convSpread, t0, alpha, s0, beta, HQ)``."""

    def __init__(self, population=4, imax=5000, iTc=20, delta=2.0, convDelay=0.75,
                 convSpread=0.15, t0=20.0, alpha=0.9, s0=100.0, beta=5.3, HQ=None, seed=0,
                 convergence=True):
        self.population = int(population)
        self.imax = int(imax)
        self.iTc = int(iTc)
        self.delta = float(np.float32(delta))
        self.convergenceDelay = float(np.float32(convDelay))
        self.convergenceRate = float(np.float32(convSpread))
        self.t0 = float(np.float32(t0))
        self.alpha = float(np.float32(alpha))
        self.s0 = float(np.float32(s0))
        self.beta = float(np.float32(beta))
        self.plugin = HQ
        self.seed = int(seed)
        self.convergence = bool(convergence)

    def getImax(self):  # SW:36
        return self.imax

    def getPopulationSize(self):  # SW:113
        return self.population

    def params(self) -> _lib.hq_swasa_params:
        return _lib.hq_swasa_params(self.population, self.imax, self.iTc, self.delta,
                                    self.convergenceDelay, self.convergenceRate, self.t0,
                                    self.alpha, self.s0, self.beta, int(self.convergence))

    def computePenalty(self, usedColors) -> float:  # SW:74-82
        return float(np.count_nonzero(np.asarray(usedColors) == 0)) * self.delta

    def search_host(self, K: int, eval_population, iterations=None):
        """Run the native SWASA driver with a Python population evaluator.

        eval_population(palettes (P, K, 4) float32) -> costs (P,).  Returns
        (best_colors float[4K], best_error, trace (iterations, 1+P)).  This is
        the hook the CPU tests use to check the policy without a GPU.
        """
        lib = load()
        params = self.params()
        iters = self.imax if iterations is None else int(iterations)
        errbox = []

        def _cb(user, pal, P, KK, costs):
            try:
                arr = np.ctypeslib.as_array(pal, shape=(P * KK * 4,)).reshape(P, KK, 4).copy()
                out = np.asarray(eval_population(arr), dtype=np.float64)
                for i in range(P):
                    costs[i] = float(out[i])
                return 0
            except Exception as e:  # surfaced after the call
                errbox.append(e)
                return 1

        cb = _lib.EVAL_FN(_cb)
        best = np.zeros(4 * K, np.float32)
        err = C.c_double()
        trace = np.zeros(iters * (1 + self.population), np.float64)
        rc = lib.hq_swasa_search_host(C.byref(params), int(K), self.seed, iters, cb, None,
                                      _lib.fptr(best), C.byref(err), _lib.dptr(trace))
        if errbox:
            raise errbox[0]
        check(rc)
        return best, err.value, trace.reshape(iters, 1 + self.population)
