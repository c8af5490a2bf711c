"""Contents of the HDF5 fixtures (shared by tests/golden/make_h5_fixture.py, which writes them
with h5py, and tests/test_h5_cpu.py, which reads them with the in-tree reader). A Keras-3
`save_weights` tree of a fine-tuned PPODiffusion at small width (hidden 32): the actor (DiffusionMLP),
actor_ft and critic (CriticObs), plus a few extra shapes/dtypes that exercise the format."""
import numpy as np

HIDDEN, TD, XD, SD, CH = 32, 16, 12, 11, 24
BLOCK = "two_layer_pre_activation_res_net_linear"


def actor_layout(prefix, h=HIDDEN):
    """Keras-3 paths of DiffusionMLP's Dense variables (keys: the flat-spec names of ops.py)."""
    return {
        "time_w1": (f"{prefix}time_embedding/layers/dense/vars/0", (TD, 2 * TD)),
        "time_b1": (f"{prefix}time_embedding/layers/dense/vars/1", (2 * TD,)),
        "time_w2": (f"{prefix}time_embedding/layers/dense_1/vars/0", (2 * TD, TD)),
        "time_b2": (f"{prefix}time_embedding/layers/dense_1/vars/1", (TD,)),
        "in_w": (f"{prefix}mlp_mean/input_layer/vars/0", (XD + TD + SD, h)),
        "in_b": (f"{prefix}mlp_mean/input_layer/vars/1", (h,)),
        "l1_w": (f"{prefix}mlp_mean/residual_blocks/{BLOCK}/l1/vars/0", (h, h)),
        "l1_b": (f"{prefix}mlp_mean/residual_blocks/{BLOCK}/l1/vars/1", (h,)),
        "l2_w": (f"{prefix}mlp_mean/residual_blocks/{BLOCK}/l2/vars/0", (h, h)),
        "l2_b": (f"{prefix}mlp_mean/residual_blocks/{BLOCK}/l2/vars/1", (h,)),
        "out_w": (f"{prefix}mlp_mean/output_layer/vars/0", (h, XD)),
        "out_b": (f"{prefix}mlp_mean/output_layer/vars/1", (XD,)),
    }


def critic_layout(prefix, h=CH):
    return {
        "in_w": (f"{prefix}Q1/input_layer/vars/0", (SD, h)), "in_b": (f"{prefix}Q1/input_layer/vars/1", (h,)),
        "l1_w": (f"{prefix}Q1/residual_blocks/{BLOCK}/l1/vars/0", (h, h)),
        "l1_b": (f"{prefix}Q1/residual_blocks/{BLOCK}/l1/vars/1", (h,)),
        "l2_w": (f"{prefix}Q1/residual_blocks/{BLOCK}/l2/vars/0", (h, h)),
        "l2_b": (f"{prefix}Q1/residual_blocks/{BLOCK}/l2/vars/1", (h,)),
        "out_w": (f"{prefix}Q1/output_layer/vars/0", (h, 1)), "out_b": (f"{prefix}Q1/output_layer/vars/1", (1,)),
    }


def fixture_arrays(many=True):
    """many=False drops the 12-child group: under libver="latest" HDF5 stores a group of more than
    8 links densely (fractal heap + v2 B-tree), which the in-tree reader rejects with a clear
    error; Keras writes with h5py's default libver (symbol tables, any size)."""
    rng = np.random.default_rng(20261016)
    arrays = {}
    for layout in (actor_layout("actor/"), actor_layout("actor_ft/"), critic_layout("critic/")):
        for _, (path, shape) in layout.items():
            arrays[path] = rng.standard_normal(shape).astype(np.float32)
    # format coverage: a float64 vector, an int32 matrix, a scalar, a 12-child group (more than
    # one symbol-table node at the default leaf K = 4), an empty group
    arrays["extra/f64"] = rng.standard_normal(7)
    arrays["extra/i32"] = rng.integers(-1000, 1000, (3, 5)).astype(np.int32)
    arrays["extra/scalar"] = np.float32(2.5)
    for i in range(12 if many else 0):
        arrays[f"extra/many/v{i:02d}"] = np.full((2,), i, np.float32)
    groups = ["vars", "actor/vars", "critic/vars", "extra/empty"]
    return arrays, groups
