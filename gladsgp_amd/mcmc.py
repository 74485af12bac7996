"""Metropolis fit of the sim-only GPMSA emulator on the GPU (SEPIA's do_mcmc / tune_step_sizes).

Reference usage replaced (``src/model.py:218-238``)::

    model.params.lamWOs = SepiaParam(val=pc_prec, name='lamWOs', val_shape=(1, 1),
        dist='Gamma', params=[50, 50/pc_prec], bounds=[1., np.inf], mcmcStepParam=10,
        mcmcStepType='Uniform')
    model.params.mcmcList = [model.params.betaU, model.params.lamUz, model.params.lamWs,
                             model.params.lamWOs]
    model.tune_step_sizes(100, 5)
    model.do_mcmc(512)

SEPIA (``timghill/SEPIA@ffe3b60``) is not available offline, so the
sampler is restated from the GPMSA model it implements; every constant below that the
reference's own files do not pin is marked *unpinned*.

Model (per principal component j = 0..P-1, one GP each, w_hat_j = PC weights of the n runs)::

    Sigma_j = (1/lamUz_j) exp(-sum_k betaU[k+1, j] (t_ik - t_i'k)^2)
              + (1/lamWs_j + 1/(lamWOs LamSim_j)) I
    loglik  = sum_j  -1/2 log|Sigma_j| - 1/2 w_hat_j^T Sigma_j^-1 w_hat_j           

betaU is (d+1, P); row 0 belongs to the dummy x input, whose differences are all zero, so it
only moves under its prior (the reference's sample layout ``(S, (d+1) P)``, C order,
``mcmc_diagnostics_advanced.py:57``).

Priors (log densities up to constants) and proposals:

  ===========  ===================================  ==========  ===========  ============
  param        prior                                bounds      step (dflt)  step type
  ===========  ===================================  ==========  ===========  ============
  betaU        Beta(1, 0.1) on rho = exp(-beta/4)   [0, inf)    0.1          BetaRho
  lamUz        Gamma(5, 5)                          [0.3, inf)  5            Uniform
  lamWs        Gamma(3, 0.003)                      [60, 1e5]   100          Uniform
  lamWOs       Gamma(5, 0.005); the reference       [60, 1e5]   100          Uniform
               overrides it with Gamma(50, 50/pc_prec), [1, inf), step 10 (model.py:225-229)
  ===========  ===================================  ==========  ===========  ============

The default step sizes are pinned by ``examples/03...ipynb:192-208``; the prior families,
parameters and bounds are the GPMSA defaults and are *unpinned*.  Gamma is (shape, rate).
Proposals: ``Uniform`` x' = x + step (u - 1/2); ``BetaRho`` the same move on rho, then
beta' = -4 log rho'.  A proposal outside the bounds is rejected.  Acceptance:
log u < log post(x') - log post(x).

Sweep (one MCMC iteration) = component-wise Metropolis over mcmcList in order: betaU row by
row, then lamUz, lamWs, lamWOs.  Given lamWOs the P GPs are independent, so the P elements of
one betaU row (or of lamUz, lamWs) are proposed together and accepted or rejected one by one:
that is the same Markov kernel as updating them one after another, evaluated as ONE batched
gp_loglik (Gram -> Cholesky -> quadratic form for the P GPs).  lamWOs touches every GP and is
accepted on the sum.  The whole sweep is stream-ordered device work: no host synchronisation,
proposals and accept/reject are device tensor ops on uniforms drawn on the host from a seeded
numpy Generator (so a CPU restatement fed the same uniforms reproduces the chain).

tune_step_sizes(n_burn, n_levels): after n_burn burn-in sweeps at the default steps, for each
level l the steps are default * 2^e_l, e_l evenly spaced in [-(n_levels-1)/2, (n_levels-1)/2];
n_burn sweeps are run at each level continuing the chain, acceptances are counted per element, and a binomial logistic regression of acceptance on
log(step) gives the step whose predicted acceptance is 1/e (logit = log(1/(e-1))), anchored by
one pseudo-acceptance far below and one pseudo-rejection far above the ladder so that a
parameter accepted (or rejected) at every level still gets an extrapolated step; the result
is clamped to the anchors' span, to 1 for BetaRho moves (rho lives in (0, 1]) and to the bound
width for a bounded parameter.  Burn-in, ladder base, target, regularisation and clamps are
*unpinned* (GPMSA's stepsize procedure).
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _capi, kernels

F64 = torch.float64
TARGET_LOGIT = math.log(1.0 / (math.e - 1.0))   # acceptance 1/e
RHO_MAX = 0.999                                  # rho clipped in the Beta prior (beta -> 0)


class SepiaParam:
    """One model parameter: value, prior and Metropolis step (SEPIA's SepiaParam surface).

    Signature as the reference calls it (``src/model.py:225-229``).
    """

    def __init__(self, val, name, val_shape, dist="Normal", params=None, bounds=None,
                 mcmcStepParam=0.1, mcmcStepType="Uniform", fixed=None):
        self.name = name
        self.val_shape = tuple(val_shape)
        self.val = np.broadcast_to(np.asarray(val, dtype=np.float64), self.val_shape).copy()
        if dist not in ("Gamma", "Beta", "Uniform", "Normal"):
            raise ValueError(f"unsupported prior {dist!r}")
        self.dist = dist
        self.params = [float(p) for p in (params if params is not None else [0.0, 1.0])]
        b = bounds if bounds is not None else [-np.inf, np.inf]
        self.bounds = (float(b[0]), float(b[1]))
        self.mcmcStepParam = np.broadcast_to(np.asarray(mcmcStepParam, dtype=np.float64),
                                             self.val_shape).copy()
        if mcmcStepType not in ("Uniform", "BetaRho"):
            raise ValueError(f"unsupported step type {mcmcStepType!r}")
        self.mcmcStepType = mcmcStepType
        self.fixed = np.zeros(self.val_shape, bool) if fixed is None else np.asarray(fixed, bool)

    def __repr__(self):
        return (f"SepiaParam({self.name}, shape={self.val_shape}, {self.dist}{self.params}, "
                f"bounds={self.bounds}, step={self.mcmcStepType})")


class ModelParams:
    """``model.params``: attributes betaU, lamUz, lamWs, lamWOs and ``mcmcList``."""

    names = ("betaU", "lamUz", "lamWs", "lamWOs")

    def __init__(self, d: int, P: int):
        # GPMSA / SEPIA defaults (step sizes pinned by 03...ipynb:192-208; the rest unpinned)
        self.betaU = SepiaParam(0.1, "betaU", (d + 1, P), "Beta", [1.0, 0.1], [0.0, np.inf],
                                0.1, "BetaRho")
        self.lamUz = SepiaParam(1.0, "lamUz", (1, P), "Gamma", [5.0, 5.0], [0.3, np.inf],
                                5.0, "Uniform")
        self.lamWs = SepiaParam(1000.0, "lamWs", (1, P), "Gamma", [3.0, 0.003], [60.0, 1e5],
                                100.0, "Uniform")
        self.lamWOs = SepiaParam(1000.0, "lamWOs", (1, 1), "Gamma", [5.0, 0.005], [60.0, 1e5],
                                 100.0, "Uniform")
        self.mcmcList = [self.betaU, self.lamUz, self.lamWs, self.lamWOs]

    def __getitem__(self, name):          # dict-style access to values
        return getattr(self, name).val

    def __setitem__(self, name, value):
        p = getattr(self, name)
        p.val = np.broadcast_to(np.asarray(value, dtype=np.float64), p.val_shape).copy()

    def values(self) -> dict:
        return {k: getattr(self, k).val.copy() for k in self.names}


# ------------------------------------------------------------------------------ priors (torch)
def log_prior(p: SepiaParam, x: torch.Tensor) -> torch.Tensor:
    """Elementwise log prior density of parameter ``p`` at values ``x`` (device tensor)."""
    a, b = p.params
    if p.dist == "Gamma":
        return (a - 1.0) * torch.log(x) - b * x
    if p.dist == "Beta":                    # on rho = exp(-x / 4)
        rho = torch.clamp(torch.exp(-x / 4.0), max=RHO_MAX)
        return (a - 1.0) * torch.log(rho) + (b - 1.0) * torch.log1p(-rho)
    if p.dist == "Normal":
        return -0.5 * ((x - a) / b) ** 2
    return torch.zeros_like(x)              # Uniform on the bounds


def propose(p: SepiaParam, x: torch.Tensor, step: torch.Tensor, u: torch.Tensor):
    """Candidate values and in-bounds mask for a Metropolis move of ``p``."""
    if p.mcmcStepType == "BetaRho":
        rho = torch.exp(-x / 4.0) + step * (u - 0.5)
        ok = (rho > 0.0) & (rho <= 1.0)
        cand = -4.0 * torch.log(torch.where(ok, rho, torch.ones_like(rho)))
    else:
        cand = x + step * (u - 0.5)
        ok = torch.ones_like(cand, dtype=torch.bool)
    lo, hi = p.bounds
    ok = ok & (cand >= lo) & (cand <= hi)
    return torch.where(ok, cand, x), ok


# --------------------------------------------------------------------------- device sampler
@dataclass
class ChainState:
    """Device-resident chain state; updated in place so a captured sweep graph stays valid."""

    betaU: torch.Tensor        # (d+1, P)
    lamUz: torch.Tensor        # (P,)
    lamWs: torch.Tensor        # (P,)
    lamWOs: torch.Tensor       # (1,)
    ll: torch.Tensor           # (P,) current per-GP log-likelihood
    acc: dict = field(default_factory=dict)   # per-element acceptance counters (device)


def uniforms_per_sweep(d: int, P: int) -> int:
    """Uniform draws one sweep consumes: (proposal, acceptance) per updated element."""
    return 2 * ((d + 1) * P + 2 * P + 1)


def default_spec(n: int, P: int, updates: int) -> int:
    """Speculative group size with the least modelled sweep time: ceil(updates / s) batched
    gp_loglik calls of (2^s - 1) P problems each, a call costing the longer of the
    factorisation's chain (~25 us per 64-column step) and its work (~4.8 us per n = 512 problem,
    scaled by n^3).  Fitted on MI355X (profiles/r06/r06al_ab_spec.log: 24 problems 0.21 ms, 56
    0.26, 120 0.58 at n = 512); it picks spec 3 at the fit's n = 512, P = 8.  Speed only: every
    spec gives the same chain."""
    def sweep(s):
        call = max(0.025 * -(-n // 64), 0.0048 * (2 ** s - 1) * P * (n / 512.0) ** 3)
        return -(-updates // s) * call
    return min(range(1, _capi.MCMC_MAX_GROUP + 1), key=sweep)


class GPUSampler:
    """Component-wise Metropolis over the P PC-GPs of one emulator, all state on the device.

    One sweep is ~11 batched gp_loglik calls plus elementwise proposal / accept work: a few
    hundred small launches.  By default (``use_graph`` None; GPFIT_MCMC_GRAPH=0 opts out) the
    sweep is captured once as a HIP graph (torch.cuda.CUDAGraph) over static buffers -- chain
    state, uniforms, step sizes, counters -- and replayed: at the timing.csv configuration
    (n = 512, P = 8) 3.75 vs 4.04-4.26 ms per sweep eager, the fit 5.0-5.4 vs 5.7-6.3 s
    (profiles/r03/ab_mcmc_graph.log; round 2 measured the opposite while the factorisation
    still allocated its scratch inside every call).  Both paths run the same in-place sweep.

    ``spec`` (default: default_spec(n, P, d + 3); GPFIT_MCMC_SPEC overrides): likelihood-
    changing updates per batched gp_loglik, evaluated speculatively for every outcome of the
    group's earlier updates (see _sweep).  At n = 512 a factorisation is latency-bound (its
    64-column chain), so evaluating 3P problems costs about what P did: spec 2 took a sweep from
    11 gp_loglik calls to 6, 3.79 -> 2.86 ms per sweep (profiles/r03/ab_mcmc_spec.log).  With
    the in-chain likelihood (round 6) 7P = 56 problems cost 0.26 ms per call against 0.21 for
    24, so spec 3 (4 calls) wins at P = 8: 1.278 -> 1.054 ms per sweep, the fit 1.67 -> 1.41-1.44
    s (profiles/r06/r06al_ab_spec.log).
    """

    def __init__(self, X: torch.Tensor, w_hat: torch.Tensor, LamSim: torch.Tensor,
                 params: ModelParams, use_graph: bool | None = None, spec: int | None = None,
                 fused: bool | None = None):
        self.X = X.contiguous()
        self.w = w_hat.contiguous()                 # (P, n)
        self.P, self.n = self.w.shape
        self.d = self.X.shape[1]
        self.dev = self.X.device
        self.lam = LamSim.to(self.dev, F64).reshape(self.P).contiguous()
        self.params = params
        self.ws = kernels.LoglikWorkspace(self.n, self.P, self.dev)
        self._beta = torch.empty((self.P, self.d), dtype=F64, device=self.dev)
        self._s = torch.empty(self.P, dtype=F64, device=self.dev)
        self._delta = torch.empty(self.P, dtype=F64, device=self.dev)
        self._ll = torch.empty(self.P, dtype=F64, device=self.dev)
        self.nu = uniforms_per_sweep(self.d, self.P)
        self.u = torch.zeros(self.nu, dtype=F64, device=self.dev)        # static uniforms
        self.steps = {k: self._t(getattr(params, k).mcmcStepParam) for k in ModelParams.names}
        # the recorded state, one flat row: betaU (d+1, P) | lamUz | lamWs | lamWOs | log post
        # (ChainState's tensors are views of it, so a sample is recorded with one copy)
        P_, d_ = self.P, self.d
        self._cols = {"betaU": (0, (d_ + 1) * P_)}
        o_ = (d_ + 1) * P_
        for k_, w_ in (("lamUz", P_), ("lamWs", P_), ("lamWOs", 1), ("logPost", 1)):
            self._cols[k_] = (o_, o_ + w_)
            o_ += w_
        self._flat = torch.zeros(o_, dtype=F64, device=self.dev)
        self.lp = self._flat[self._cols["logPost"][0]:]                 # log posterior
        if use_graph is None:
            use_graph = os.environ.get("GPFIT_MCMC_GRAPH", "1") == "1"
        self.use_graph = use_graph and self.dev.type == "cuda"
        self.graph = None
        # sweeps per replayed graph in run() (GPFIT_MCMC_BLOCK; 1: one sweep per replay)
        self.block = max(1, int(os.environ.get("GPFIT_MCMC_BLOCK", "16")))
        # decide + next prep in one launch (gp_mcmc_group_step); GPFIT_MCMC_MERGE=0: two
        self._merge = os.environ.get("GPFIT_MCMC_MERGE", "1") == "1"
        self._bgraph = {}
        self.st = None
        if spec is None:
            spec = int(os.environ.get("GPFIT_MCMC_SPEC", "0")) or default_spec(self.n, self.P,
                                                                               self.d + 3)
        if spec < 1:
            raise ValueError("spec (updates per speculative group) must be >= 1")
        # the likelihood-changing updates of a sweep, in mcmcList order (betaU row 0, the
        # dummy x, moves under its prior alone)
        ups = [("betaU", k) for k in range(1, self.d + 1)] + [(nm, None) for nm in
                                                               ("lamUz", "lamWs", "lamWOs")]
        self.groups = [ups[i:i + spec] for i in range(0, len(ups), spec)]
        self.spec = spec
        if fused is None:
            fused = os.environ.get("GPFIT_MCMC_FUSED", "1") == "1"
        self.fused = fused and self.dev.type == "cuda"
        if self.fused and spec > _capi.MCMC_MAX_GROUP:
            raise ValueError(f"spec > {_capi.MCMC_MAX_GROUP} needs fused=False")
        self._S = None
        self._scratch = torch.zeros(3 * _capi.MCMC_MAX_GROUP * self.P, dtype=F64, device=self.dev)
        self._gbuf = {}
        for g in self.groups:
            sets = 2 ** len(g) - 1
            if sets not in self._gbuf:
                B = sets * self.P
                self._gbuf[sets] = dict(
                    ws=self.ws if B == self.P else kernels.LoglikWorkspace(self.n, B, self.dev),
                    beta=torch.empty((B, self.d), dtype=F64, device=self.dev),
                    s=torch.empty(B, dtype=F64, device=self.dev),
                    delta=torch.empty(B, dtype=F64, device=self.dev),
                    ll=torch.empty(B, dtype=F64, device=self.dev),
                    w=self.w.repeat(sets, 1).contiguous())

    def _t(self, a) -> torch.Tensor:
        return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64), device=self.dev)

    # -- state ---------------------------------------------------------------------------
    def init_state(self) -> ChainState:
        """Chain state from params' current values (allocated once; later calls copy)."""
        pr = self.params
        vals = (self._t(pr.betaU.val), self._t(pr.lamUz.val).reshape(self.P),
                self._t(pr.lamWs.val).reshape(self.P), self._t(pr.lamWOs.val).reshape(1))
        if self.st is None:
            z = torch.zeros(self.P, dtype=F64, device=self.dev)
            views = []
            for k, v in zip(("betaU", "lamUz", "lamWs", "lamWOs"), vals):
                a, b = self._cols[k]
                t = self._flat[a:b].view(v.shape)
                t.copy_(v)
                views.append(t)
            self.st = ChainState(*views, z.clone())
            # one (d + 4, P) block indexed by update code (gp_mcmc_state.acc), viewed per update
            d = self.d
            self._acc = torch.zeros((d + 4, self.P), dtype=F64, device=self.dev)
            self.st.acc = {("betaU", k): self._acc[k] for k in range(d + 1)}
            self.st.acc.update({"lamUz": self._acc[d + 1], "lamWs": self._acc[d + 2],
                                "lamWOs": self._acc[d + 3, :1]})
        else:
            for t, v in zip((self.st.betaU, self.st.lamUz, self.st.lamWs, self.st.lamWOs),
                            vals):
                t.copy_(v)
        self.st.ll.copy_(self.loglik(self.st.betaU, self.st.lamUz, self.st.lamWs,
                                     self.st.lamWOs))
        self.reset_counts()
        return self.st

    def reset_counts(self) -> None:
        for c in self.st.acc.values():
            c.zero_()

    def counts(self) -> dict:
        return {k: v.cpu().numpy() for k, v in self.st.acc.items()}

    def set_steps(self, scale: float = 1.0) -> None:
        for k in ModelParams.names:
            self.steps[k].copy_(self._t(getattr(self.params, k).mcmcStepParam * scale))

    def write_back(self) -> None:
        pr, st = self.params, self.st
        pr.betaU.val = st.betaU.cpu().numpy().reshape(pr.betaU.val_shape)
        pr.lamUz.val = st.lamUz.cpu().numpy().reshape(pr.lamUz.val_shape)
        pr.lamWs.val = st.lamWs.cpu().numpy().reshape(pr.lamWs.val_shape)
        pr.lamWOs.val = st.lamWOs.cpu().numpy().reshape(pr.lamWOs.val_shape)

    # -- likelihood / posterior ----------------------------------------------------------
    def loglik(self, betaU, lamUz, lamWs, lamWOs) -> torch.Tensor:
        """Per-GP log-likelihood (P,) for the given parameters (one gp_loglik call)."""
        self._beta.copy_(betaU[1:].transpose(0, 1))
        torch.reciprocal(lamUz, out=self._s)
        torch.add(torch.reciprocal(lamWs), torch.reciprocal(lamWOs * self.lam), out=self._delta)
        return kernels.loglik(self.X, self._beta, self._s, self._delta, self.w, self.ws,
                              out=self._ll)

    def log_post(self) -> torch.Tensor:
        pr, st = self.params, self.st
        lp = st.ll.sum()
        lp = lp + log_prior(pr.betaU, st.betaU).sum() + log_prior(pr.lamUz, st.lamUz).sum()
        lp = lp + log_prior(pr.lamWs, st.lamWs).sum() + log_prior(pr.lamWOs, st.lamWOs).sum()
        return lp

    # -- one sweep -----------------------------------------------------------------------
    def _fill(self, buf: dict, slot: int, st: dict) -> None:
        """Model inputs (beta, s, delta) of the P GPs at parameter state ``st`` into rows
        slot P .. (slot + 1) P of a speculative group's batch."""
        sl = slice(slot * self.P, (slot + 1) * self.P)
        buf["beta"][sl].copy_(st["betaU"][1:].transpose(0, 1))
        torch.reciprocal(st["lamUz"], out=buf["s"][sl])
        torch.add(torch.reciprocal(st["lamWs"]), torch.reciprocal(st["lamWOs"] * self.lam),
                  out=buf["delta"][sl])

    @staticmethod
    def _with(st: dict, u, cand) -> dict:
        """Parameter state ``st`` with update ``u``'s element(s) set to ``cand``."""
        name, k = u
        out = dict(st)
        if name == "betaU":
            b = st["betaU"].clone()
            b[k] = cand
            out["betaU"] = b
        else:
            out[name] = cand
        return out

    def _propose(self, u, take):
        pr, st, steps, P = self.params, self.st, self.steps, self.P
        name, k = u
        p = getattr(pr, name)
        if name == "betaU":
            cur, step, m = st.betaU[k], steps["betaU"][k], P
        elif name == "lamWOs":
            cur, step, m = st.lamWOs, steps["lamWOs"].reshape(1), 1
        else:
            cur, step, m = getattr(st, name), steps[name].reshape(P), P
        up, ua = take(m), take(m)
        cand, ok = propose(p, cur, step, up)
        return cand, ok, log_prior(p, cand) - log_prior(p, cur), ua, cur

    def _accept(self, u, prop, ll_new) -> torch.Tensor:
        """Metropolis decision for update ``u`` given the proposal's per-GP likelihood."""
        st = self.st
        cand, ok, dlp, ua, cur = prop
        name, k = u
        if name == "lamWOs":                 # shared by every GP: accepted on the sum
            acc = ok & (torch.log(ua) < (ll_new - st.ll).sum() + dlp.sum())
        else:
            acc = ok & (torch.log(ua) < ll_new - st.ll + dlp)
        cur.copy_(torch.where(acc, cand, cur))
        st.ll.copy_(torch.where(acc, ll_new, st.ll))
        st.acc[("betaU", k) if name == "betaU" else name].add_(acc.to(F64))
        return acc

    def _code(self, u) -> int:
        name, k = u
        return k if name == "betaU" else self.d + {"lamUz": 1, "lamWs": 2, "lamWOs": 3}[name]

    def _state_struct(self) -> "_capi.McmcState":
        """gp_mcmc_state over the static buffers and the current priors."""
        st, pr = self.st, self.params
        S = _capi.McmcState()
        for nm, t in (("betaU", st.betaU), ("lamUz", st.lamUz), ("lamWs", st.lamWs),
                      ("lamWOs", st.lamWOs), ("ll", st.ll), ("lam", self.lam), ("u", self.u),
                      ("step_betaU", self.steps["betaU"]), ("step_lamUz", self.steps["lamUz"]),
                      ("step_lamWs", self.steps["lamWs"]), ("step_lamWOs", self.steps["lamWOs"]),
                      ("acc", self._acc), ("lp", self.lp), ("scratch", self._scratch)):
            if not t.is_contiguous() or t.dtype != F64:
                raise TypeError(f"mcmc state buffer {nm} must be contiguous float64")
            setattr(S, nm, t.data_ptr())
        S.P, S.d = self.P, self.d
        for i, nm in enumerate(ModelParams.names):
            p = getattr(pr, nm)
            S.dist[i] = _capi.MCMC_DIST[p.dist]
            S.steptype[i] = _capi.MCMC_STEP[p.mcmcStepType]
            S.pa[i], S.pb[i] = p.params
            S.lo[i], S.hi[i] = p.bounds
        return S

    def _sweep(self) -> None:
        if self.fused:
            self._sweep_fused()
        else:
            self._sweep_torch()

    def _sweep_fused(self) -> None:
        """The sweep of _sweep_torch with each speculative group's proposals and decisions in
        single-workgroup kernels around its gp_loglik (csrc/mcmc.hip): the first group's
        gp_mcmc_group_prep, then after each gp_loglik one gp_mcmc_group_step (this group's
        decisions + the next group's proposals; gp_mcmc_group_decide after the last), so
        2 + gp_loglik's launches per group instead of ~100."""
        self._S = self._state_struct()          # kept alive: the library reads it per call
        S = ctypes.addressof(self._S)
        stream = kernels._stream(self.dev)
        last = len(self.groups) - 1
        kinds = [(ctypes.c_int * len(g))(*[self._code(u) for u in g]) for g in self.groups]
        self._kinds = kinds                     # (kept alive with _S)
        bufs = [self._gbuf[2 ** len(g) - 1] for g in self.groups]
        b0 = bufs[0]
        _capi.call("gp_mcmc_group_prep", S, ctypes.addressof(kinds[0]), len(self.groups[0]), 1,
                   b0["beta"].data_ptr(), b0["s"].data_ptr(), b0["delta"].data_ptr(), stream)
        for gi, grp in enumerate(self.groups):
            buf = bufs[gi]
            kernels.loglik(self.X, buf["beta"], buf["s"], buf["delta"], buf["w"], buf["ws"],
                           out=buf["ll"])
            if gi == last or not self._merge:
                _capi.call("gp_mcmc_group_decide", S, ctypes.addressof(kinds[gi]), len(grp),
                           int(gi == last), buf["ll"].data_ptr(), stream)
                if gi < last:
                    nb = bufs[gi + 1]
                    _capi.call("gp_mcmc_group_prep", S, ctypes.addressof(kinds[gi + 1]),
                               len(self.groups[gi + 1]), 0, nb["beta"].data_ptr(),
                               nb["s"].data_ptr(), nb["delta"].data_ptr(), stream)
            else:
                nb = bufs[gi + 1]
                _capi.call("gp_mcmc_group_step", S, ctypes.addressof(kinds[gi]), len(grp), 0,
                           buf["ll"].data_ptr(), S, ctypes.addressof(kinds[gi + 1]),
                           len(self.groups[gi + 1]), 0, nb["beta"].data_ptr(),
                           nb["s"].data_ptr(), nb["delta"].data_ptr(), stream)

    def _sweep_torch(self) -> None:
        """One component-wise Metropolis sweep on the static buffers (graph-capturable: no
        allocation that outlives it, no host synchronisation, in-place state updates), as
        tensor ops (the host-logic reference of the fused sweep; runs on any device).

        Speculative groups: the updates u_1 .. u_g of a group are proposed together and ONE
        batched gp_loglik evaluates, for every i, u_i's proposal at each of the 2^(i-1)
        accept/reject outcomes of u_1 .. u_i-1 (2^g - 1 parameter states x P GPs); the
        decisions are then taken in order, each reading the likelihood of the outcome that
        actually happened (per GP: the P GPs are independent given lamWOs, whose decision is
        one for all).  Proposals, uniforms and decisions are those of the one-update-at-a-time
        sweep, so the chain is the same Markov chain, draw for draw; what changes is that the
        factorisations, whose latency (a 64-column chain step per tile) bounds a sweep at
        n = 512, are issued g at a time (spec = 1: one call per update)."""
        pr, st, P, u = self.params, self.st, self.P, self.u
        o = 0

        def take(k):
            nonlocal o
            r = u[o:o + k]
            o += k
            return r

        # betaU row 0 (the dummy x): the likelihood does not depend on it
        cand, ok, dlp, ua, cur = self._propose(("betaU", 0), take)
        acc = ok & (torch.log(ua) < dlp)
        cur.copy_(torch.where(acc, cand, cur))
        st.acc[("betaU", 0)].add_(acc.to(F64))
        for grp in self.groups:
            props = [self._propose(g, take) for g in grp]
            buf = self._gbuf[2 ** len(grp) - 1]
            s0 = {"betaU": st.betaU, "lamUz": st.lamUz, "lamWs": st.lamWs, "lamWOs": st.lamWOs}
            slot, base = 0, []
            for i, g in enumerate(grp):
                base.append(slot)
                for pat in range(2 ** i):         # outcome pattern of the group's earlier updates
                    sx = s0
                    for j in range(i):
                        if (pat >> j) & 1:
                            sx = self._with(sx, grp[j], props[j][0])
                    self._fill(buf, slot, self._with(sx, g, props[i][0]))
                    slot += 1
            ll_all = kernels.loglik(self.X, buf["beta"], buf["s"], buf["delta"], buf["w"],
                                    buf["ws"], out=buf["ll"]).view(-1, P)
            pat = None
            for i, g in enumerate(grp):
                ll_i = ll_all[base[i]:base[i] + 2 ** i]
                ll_new = ll_i[0] if pat is None else ll_i.gather(0, pat.view(1, P)).view(P)
                acc = self._accept(g, props[i], ll_new).expand(P).long() << i
                pat = acc if pat is None else pat + acc
        self.lp.copy_(self.log_post().reshape(1))

    def _capture(self) -> None:
        """Record one sweep as a graph (capture does not execute it: the chain is untouched)."""
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._sweep()
        self.graph = g

    def sweep(self) -> None:
        if self.use_graph:
            if self.graph is None:
                self._capture()
            self.graph.replay()
        else:
            self._sweep()

    def _capture_block(self, record: bool) -> None:
        """Record ``block`` sweeps as one graph: sweep j reads the uniforms of row j of a static
        block and (``record``) copies the flat state into row j of a static record block.  One
        replay per block instead of one per sweep, and one copy per recorded sample instead of
        one uniform upload + five record copies.  Fit: 1.368 ms per sweep at 16 sweeps per replay
        vs 1.373-1.375 at one (the flat one-copy record in both), 1.374-1.383 at 32
        (profiles/r05/r05_block_fit.log): the host keeps the queue full either way."""
        B = self.block
        if not hasattr(self, "_ublk"):
            self._ublk = torch.zeros((B, self.nu), dtype=F64, device=self.dev)
            self._rblk = torch.zeros((B, self._flat.numel()), dtype=F64, device=self.dev)
        torch.cuda.synchronize(self.dev)
        g = torch.cuda.CUDAGraph()
        u0 = self.u
        try:
            with torch.cuda.graph(g):
                for j in range(B):
                    self.u = self._ublk[j]
                    self._sweep()
                    if record:
                        self._rblk[j].copy_(self._flat)
        finally:
            self.u = u0
        self._bgraph[record] = g

    # -- chains --------------------------------------------------------------------------
    def run(self, nsamp: int, rng: np.random.Generator, record: bool = True, block: int = 64):
        """``nsamp`` sweeps from the current state (init_state() first if there is none);
        returns the samples dict (numpy) when ``record``."""
        if self.st is None:
            self.init_state()
        if record:
            rec = torch.empty((nsamp, self._flat.numel()), dtype=F64, device=self.dev)
        B = self.block if self.use_graph and self.block > 1 else 0
        for a in range(0, nsamp, block):
            b = min(nsamp, a + block)
            U = self._t(rng.random((b - a, self.nu)))
            i = a
            while B and b - i >= B:                     # whole graph blocks
                if record not in self._bgraph:
                    self._capture_block(record)
                self._ublk.copy_(U[i - a:i - a + B])
                self._bgraph[record].replay()
                if record:
                    rec[i:i + B].copy_(self._rblk)
                i += B
            for i in range(i, b):                       # the rest one sweep at a time
                self.u.copy_(U[i - a])
                self.sweep()
                if record:
                    rec[i].copy_(self._flat)
        # one host check per run: a factorisation that gave up (info = -1) would otherwise be a
        # silently rejected proposal (ll = NaN); a non-PD proposal (ll = -inf) is a rejection
        for ws in {id(w): w for w in [self.ws] + [b["ws"] for b in self._gbuf.values()]}.values():
            ws.check_status()
        if not record:
            return None
        rec = rec.cpu().numpy()
        return {k: rec[:, a:b].copy() for k, (a, b) in self._cols.items()}


# --------------------------------------------------------------------------- step tuning
def logistic_step(log_steps: np.ndarray, accepts: np.ndarray, trials: int,
                  target_logit: float = TARGET_LOGIT, pseudo: float = 0.5,
                  anchor: float = math.log(100.0)) -> float:
    """Step whose fitted acceptance probability hits the target: binomial logit regression of
    acceptance on log step (IRLS).  ``pseudo`` successes/failures per level keep the fit
    finite when a level accepts everything or nothing, and two anchor observations (one
    acceptance at ``anchor`` below the smallest step, one rejection ``anchor`` above the
    largest) give the fit a slope when every level accepts (or rejects) almost always, so it
    extrapolates instead of stalling at the ladder's end.  Returns exp(log step*)."""
    xl = np.asarray(log_steps, dtype=np.float64)
    x = np.concatenate([xl, [xl.min() - anchor, xl.max() + anchor]])
    yk = np.concatenate([np.asarray(accepts, dtype=np.float64) + pseudo, [1.0, 0.0]])
    nk = np.concatenate([np.full(len(xl), float(trials) + 2.0 * pseudo), [1.0, 1.0]])
    A = np.stack([np.ones_like(x), x], axis=1)
    bvec = np.zeros(2)
    for _ in range(100):
        eta = A @ bvec
        p = 1.0 / (1.0 + np.exp(-eta))
        wgt = nk * p * (1.0 - p)
        grad = A.T @ (yk - nk * p)
        H = A.T @ (A * wgt[:, None])
        try:
            dlt = np.linalg.solve(H, grad)
        except np.linalg.LinAlgError:
            break
        bvec = bvec + dlt
        if np.max(np.abs(dlt)) < 1e-10:
            break
    b0, b1 = bvec
    if not np.all(np.isfinite(bvec)) or b1 >= -1e-12:
        rate = (yk / nk)[: len(xl)]
        return float(np.exp(xl[int(np.argmin(np.abs(rate - 1.0 / math.e)))]))
    return float(np.exp((target_logit - b0) / b1))


def tune_step_sizes(sampler: GPUSampler, n_burn: int, n_levels: int,
                    rng: np.random.Generator) -> None:
    """GPMSA-style step-size tuning (see module doc); updates params' mcmcStepParam in place
    and leaves the sampler's chain at the state reached."""
    pr = sampler.params
    if sampler.st is None:
        sampler.init_state()
    ex = np.linspace(-(n_levels - 1) / 2.0, (n_levels - 1) / 2.0, n_levels)
    base = {k: getattr(pr, k).mcmcStepParam.copy() for k in ModelParams.names}
    # burn-in at the default steps first: acceptance counted while the chain is still
    # travelling from the start values would make the smallest-step level look worst
    sampler.set_steps(1.0)
    sampler.run(n_burn, rng, record=False)
    counts = []
    for e in ex:
        sampler.set_steps(2.0 ** e)
        sampler.reset_counts()
        sampler.run(n_burn, rng, record=False)
        counts.append(sampler.counts())
    logs = {k: np.log(base[k][None] * (2.0 ** ex).reshape((-1,) + (1,) * base[k].ndim))
            for k in base}
    P, d = sampler.P, sampler.d
    new = {k: base[k].copy() for k in base}

    def fit(name, x, acc):
        # clamp: the anchors' span, rho's range for BetaRho moves, the bound width
        p = getattr(pr, name)
        st_ = logistic_step(x, acc, n_burn)
        lo_c, hi_c = math.exp(x.min() - math.log(100.0)), math.exp(x.max() + math.log(100.0))
        if p.mcmcStepType == "BetaRho":
            hi_c = min(hi_c, 1.0)
        elif np.isfinite(p.bounds[0]) and np.isfinite(p.bounds[1]):
            hi_c = min(hi_c, p.bounds[1] - p.bounds[0])
        return float(np.clip(st_, lo_c, max(hi_c, lo_c)))

    for k in range(d + 1):
        for j in range(P):
            acc = np.array([c[("betaU", k)][j] for c in counts])
            new["betaU"][k, j] = fit("betaU", logs["betaU"][:, k, j], acc)
    for name in ("lamUz", "lamWs"):
        for j in range(P):
            acc = np.array([c[name][j] for c in counts])
            new[name][0, j] = fit(name, logs[name][:, 0, j], acc)
    acc = np.array([c["lamWOs"][0] for c in counts])
    new["lamWOs"][0, 0] = fit("lamWOs", logs["lamWOs"][:, 0, 0], acc)
    for k in base:
        getattr(pr, k).mcmcStepParam = new[k]
    sampler.set_steps(1.0)
    sampler.reset_counts()
    sampler.last_tune = {"scales": 2.0 ** ex, "trials": n_burn, "base": base, "new": new,
                         "accepts": {
                             "betaU": np.array([[c[("betaU", k)] for k in range(d + 1)]
                                                for c in counts]),
                             "lamUz": np.array([c["lamUz"] for c in counts]),
                             "lamWs": np.array([c["lamWs"] for c in counts]),
                             "lamWOs": np.array([c["lamWOs"] for c in counts])}}
