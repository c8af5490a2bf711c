"""SinusoidalPosEmb (reference model/diffusion/modules.py:4-15), host form; the kernels compute the
same table in fp32 for the K (or K') distinct denoising steps."""
import math

import numpy as np


def sinusoidal_pos_emb(t, dim):
    half = dim // 2
    freqs = np.exp(np.arange(half, dtype=np.float32) * -(math.log(10000) / (half - 1)))
    e = np.asarray(t, np.float32)[:, None] * freqs[None, :]
    return np.concatenate([np.sin(e), np.cos(e)], axis=-1)
