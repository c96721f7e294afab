"""ORACLE — TEST INFRASTRUCTURE ONLY.

Deterministic, platform-independent parameters for golden fixtures: every
state_dict entry is drawn from numpy's PCG64 seeded by (seed, crc32(key)), so
a fixture stores only the seed and the key -> shape manifest.
"""
import zlib

import numpy as np

# GaussianDiffusion schedule buffers (diffusion.py:104-145) keep their values.
SCHEDULE_BUFFERS = {
    "betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_alphas_cumprod",
    "sqrt_one_minus_alphas_cumprod", "log_one_minus_alphas_cumprod",
    "sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod", "posterior_variance",
    "posterior_log_variance_clipped", "posterior_mean_coef1", "posterior_mean_coef2",
}


def _is_bn(key, shapes):
    # BatchNorm1d entries sit next to a running_mean
    base = key.rsplit(".", 1)[0]
    return (base + ".running_mean") in shapes


def seeded_value(key, shape, seed, shapes):
    rng = np.random.default_rng([seed, zlib.crc32(key.encode())])
    leaf = key.rsplit(".", 1)[-1]
    if leaf == "running_mean":
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if leaf == "running_var":
        return (1.0 + 0.3 * rng.random(shape)).astype(np.float32)
    if _is_bn(key, shapes):
        if leaf == "weight":
            return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
        return (0.1 * rng.standard_normal(shape)).astype(np.float32)
    if "lstm" in key and (leaf.startswith("weight_") or leaf.startswith("bias_")):
        hkey = key.replace("weight_ih", "weight_hh").replace("bias_ih", "weight_hh") \
                  .replace("bias_hh", "weight_hh")
        H = shapes[hkey][1] if hkey in shapes else shape[0] // 4
        k = 1.0 / np.sqrt(H)
        return rng.uniform(-k, k, shape).astype(np.float32)
    if leaf == "gamma":  # LayerNorm scale of the Transformer encoder (encoder.py:15)
        return (1.0 + 0.1 * rng.standard_normal(shape)).astype(np.float32)
    if key.endswith("emb.weight"):
        return (0.3 * rng.standard_normal(shape)).astype(np.float32)
    if len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        return (rng.standard_normal(shape) / np.sqrt(fan_in)).astype(np.float32)
    return (0.1 * rng.standard_normal(shape)).astype(np.float32)


def seeded_state_dict(shapes, seed):
    """shapes: ordered {key: tuple}; returns {key: np.ndarray} for trainable-like entries."""
    out = {}
    for key, shape in shapes.items():
        leaf = key.rsplit(".", 1)[-1]
        if leaf in SCHEDULE_BUFFERS or leaf == "num_batches_tracked":
            continue
        out[key] = seeded_value(key, tuple(shape), seed, shapes)
    return out
