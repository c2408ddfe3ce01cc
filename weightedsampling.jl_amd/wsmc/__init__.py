"""wsmc — MI355X-native SMC inner loop for WeightedSampling.jl.

The hot path (per-particle log-density accumulation, exp_norm + ESS, stratified /
systematic resampling with ancestor indices, autoRW Metropolis–Hastings moves) runs as
hand-written gfx950 HIP kernels in ``libwsmc.so`` behind the C ABI of include/wsmc.h.
This package is the host-side mirror of the reference's operator interface; it has no
CPU compute path.
"""
from . import abi
from .abi import (PROPOSAL_AUTORW, PROPOSAL_RW, RESAMPLE_MULTINOMIAL, RESAMPLE_STRATIFIED, RESAMPLE_SYSTEMATIC, WSMCError,
                  load_library)
from .context import Context, device_count
from .dsl import (Bernoulli, BernoulliLogit, Cauchy, Col, Exponential, Expr, Fx, Geometric, Gumbel, HalfNormal, Kernel,
                  Laplace, Logistic, LogNormal, MvNormal, Normal, Oscillator, Rayleigh, Uniform)
from . import dsl
from . import models
from .transformers import (Assign, Cond, FusedSSM2D, HipColumnStore, ImportanceKernel, Loop, Move, Observe,
                           Resample, RW, Sample, Sequence, SMCState, Weight, apply, autoRW, dataframe, describe,
                           expectation, importance_kernel, marginal_diversity, resampled, run, sample, score_logpdf)

__all__ = ["abi", "dsl", "Context", "device_count", "Col", "Expr", "Fx", "Bernoulli", "BernoulliLogit", "Cauchy", "Exponential", "Geometric", "Gumbel",
           "Laplace", "Logistic", "LogNormal", "Rayleigh", "Kernel", "Normal", "MvNormal", "HalfNormal",
           "Uniform", "Oscillator", "models", "load_library", "WSMCError", "RESAMPLE_STRATIFIED",
           "RESAMPLE_SYSTEMATIC", "RESAMPLE_MULTINOMIAL", "PROPOSAL_RW", "PROPOSAL_AUTORW", "Assign", "Cond", "FusedSSM2D",
           "HipColumnStore", "ImportanceKernel", "Loop", "Move", "Observe", "Resample", "RW", "Sample", "Sequence",
           "SMCState", "Weight", "apply", "autoRW", "describe", "expectation", "importance_kernel", "marginal_diversity", "resampled", "run",
           "score_logpdf", "sample", "dataframe"]
