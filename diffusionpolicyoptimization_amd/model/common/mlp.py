"""Residual MLP parameter containers (reference model/common/mlp.py:95-206).

On MI355X the MLP has no per-layer Python objects: its weights are one flat fp32 buffer in the
Keras layout (include/dppo.h) that the HIP kernels consume through a packed fragment image. These
classes hold the configuration, validate it against what the kernels implement, and create the
seeded Keras-style initialisation (glorot_uniform kernels, zero biases)."""
import math

import numpy as np

SUPPORTED_ACTIVATIONS = ("ReLU", "Mish")


def glorot_uniform(rng, fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))
    return rng.uniform(-lim, lim, size=(fan_in, fan_out)).astype(np.float32)


class ResidualMLP:
    """dims [in, h, h, h, out]: in-Dense, ONE pre-activation two-Dense block (mlp.py:121-129), out-Dense."""

    def __init__(self, dim_list, activation_type="Mish", out_activation_type="Identity", use_layernorm=False,
                 use_layernorm_final=False, dropout=0):
        dim_list = list(dim_list)
        if len(dim_list) != 5 or not (dim_list[1] == dim_list[2] == dim_list[3]):
            raise NotImplementedError(f"ResidualMLP {dim_list}: the kernels implement [in, h, h, h, out] "
                                      "(one residual block), the shape every fine-tune cfg uses")
        if use_layernorm or use_layernorm_final or dropout:
            raise NotImplementedError("layernorm/dropout are not used by the fine-tune cfgs and not implemented")
        if out_activation_type != "Identity":
            raise NotImplementedError("out_activation_type must be Identity")
        if activation_type not in SUPPORTED_ACTIVATIONS:
            raise NotImplementedError(f"activation {activation_type} not implemented")
        self.dim_list = dim_list
        self.activation_type = activation_type

    @property
    def hidden(self):
        return self.dim_list[1]

    def init_params(self, rng, prefix=""):
        i, h, o = self.dim_list[0], self.dim_list[1], self.dim_list[-1]
        return {prefix + "in_w": glorot_uniform(rng, i, h), prefix + "in_b": np.zeros(h, np.float32),
                prefix + "l1_w": glorot_uniform(rng, h, h), prefix + "l1_b": np.zeros(h, np.float32),
                prefix + "l2_w": glorot_uniform(rng, h, h), prefix + "l2_b": np.zeros(h, np.float32),
                prefix + "out_w": glorot_uniform(rng, h, o), prefix + "out_b": np.zeros(o, np.float32)}


class MLP:
    """Plain MLP (mlp.py:35-92) — only reachable from cfgs with residual_style: False, which the
    kernels do not implement; kept as a loud error rather than a silent fallback."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("non-residual MLP heads are not implemented by the MI355X kernels")
