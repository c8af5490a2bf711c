"""ctypes binding of libdppo_hip.so (include/dppo.h).

The product path has exactly one compute backend: the gfx950 HIP library built in-tree at
diffusionpolicyoptimization_amd/lib/libdppo_hip.so. There is no CPU fallback; a missing library
raises at import-of-use time with the build command.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime first so the library binds to the same one)

_HERE = os.path.dirname(os.path.abspath(__file__))
# DPPO_LIB selects a tuning build (tools/variant_build.sh); it must exist like the default one
LIB_PATH = os.environ.get("DPPO_LIB") or os.path.join(_HERE, "lib", "libdppo_hip.so")

DPPO_F32, DPPO_BF16, DPPO_F16 = 0, 1, 2
DPPO_ADAMW_KERAS, DPPO_ADAMW_TORCH = 0, 1
DPPO_STEP_DEFER_SAMPLER_TABLES = 0x100   # OR'd into dppo_optimizer_step's mode (ABI 7)
DPPO_STEP_L2_FROM_PL2 = 0x200            # (ABI 8) the actor's l2 gradient arrives factored
DPPO_PPO_L2_DEFERRED = 1                 # dppo_ppo_hparams.flags (ABI 8)
DPPO_PPO_LEARN_ETA = 2                   # (ABI 9) d loss / d eta into metrics[8]
DPPO_STEP_FUSED_PACK = 0x400             # (ABI 11) AdamW + the image in one launch
DPPO_STEP_CLEAR_GRADS = 0x800            # (ABI 11) the step zeroes the range's gradients after reading
DPPO_PPO_PRECLEARED = 4                  # (ABI 11) the part's accumulators are already zero
SCHED_COLS = 8
PRECISION = {"fp32": DPPO_F32, "f32": DPPO_F32, "bf16": DPPO_BF16, "fp16": DPPO_F16, "f16": DPPO_F16}


class DppoDims(ctypes.Structure):
    _fields_ = [("obs_dim", ctypes.c_int32), ("action_dim", ctypes.c_int32), ("horizon_steps", ctypes.c_int32),
                ("cond_steps", ctypes.c_int32), ("time_dim", ctypes.c_int32), ("actor_hidden", ctypes.c_int32),
                ("critic_hidden", ctypes.c_int32), ("denoising_steps", ctypes.c_int32),
                ("ft_denoising_steps", ctypes.c_int32), ("time_stride", ctypes.c_int32)]


class DppoPpoHparams(ctypes.Structure):
    _fields_ = [("gamma_denoising", ctypes.c_float), ("clip_ploss_coef", ctypes.c_float),
                ("clip_ploss_coef_base", ctypes.c_float), ("clip_ploss_coef_rate", ctypes.c_float),
                ("min_logprob_std", ctypes.c_float), ("vf_coef", ctypes.c_float), ("norm_adv", ctypes.c_int32),
                ("reward_horizon", ctypes.c_int32), ("loss_scale", ctypes.c_float), ("global_rows", ctypes.c_int32),
                ("flags", ctypes.c_int32), ("clip_vloss_coef", ctypes.c_float), ("old_values", ctypes.c_void_p)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_F = ctypes.c_float
_D = ctypes.c_double
_SZ = ctypes.c_size_t
_DIMS = ctypes.POINTER(DppoDims)

_SIGNATURES = {
    "dppo_abi_version": (_I, []),
    "dppo_last_error": (ctypes.c_char_p, []),
    "dppo_actor_param_count": (_SZ, [_DIMS]),
    "dppo_critic_param_count": (_SZ, [_DIMS]),
    "dppo_actor_packed_bytes": (_SZ, [_DIMS, _I]),
    "dppo_critic_packed_bytes": (_SZ, [_DIMS, _I]),
    "dppo_pack_actor": (_I, [_DIMS, _I, _P, _P, _P]),
    "dppo_pack_critic": (_I, [_DIMS, _I, _P, _P, _P]),
    "dppo_sample": (_I, [_DIMS, _I, _P, _P, _P, _P, _I, _P, _P, _U64, _U64, _I, _I, _F, _F, _F, _P, _P, _P]),
    "dppo_sample_step": (_I, [_DIMS, _I, _P, _P, _P, _P, _P, _I, _U64, _U64, _I, _I, _F, _F, _F, _P, _P, _P, _I, _P]),
    "dppo_host_alloc": (_I, [_SZ, ctypes.POINTER(ctypes.c_void_p)]),
    "dppo_host_free": (_I, [_P]),
    "dppo_rollout_enqueue": (_I, [_DIMS, _I, _P, _P, _P, _P, _P, _I, _U64, _U64, _I, _I, _F, _F, _F, _P, _P, _P, _P,
                                  ctypes.c_uint32, _P, _P]),
    "dppo_rollout_enqueue_tagged": (_I, [_DIMS, _I, _P, _P, _P, _P, _P, _I, _U64, _U64, _I, _I, _F, _F, _F, _P, _P,
                                         _P, ctypes.c_uint32, _P, _P]),
    "dppo_sampler_stream_bytes": (_I, [_DIMS, _I, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int)]),
    "dppo_sampler_layout": (_I, [_DIMS, _I, _I, ctypes.POINTER(ctypes.c_int)]),
    "dppo_sampler_max_in_flight": (_I, [_DIMS, _I, _I, ctypes.POINTER(ctypes.c_int)]),
    "dppo_sampler_plan": (_I, [_DIMS, _I, _I, ctypes.POINTER(ctypes.c_int)]),
    "dppo_sampler_release_stream": (_I, [_P]),
    "dppo_kernel_timing": (_I, [_I]),
    "dppo_kernel_timing_name": (ctypes.c_char_p, [_I]),
    "dppo_kernel_timing_read": (_I, [_I, _P, _P]),
    "dppo_logprob": (_I, [_DIMS, _I, _P, _P, _P, _P, _I, _F, _I, _P, _P, _P]),
    "dppo_critic_forward": (_I, [_DIMS, _I, _P, _P, _I, _P, _P]),
    "dppo_reward_scale_workspace_doubles": (_SZ, [_I, _I]),
    "dppo_reward_scale": (_I, [_P, _P, _P, _P, _P, _I, _I, _D, _D, _D, _P]),
    "dppo_reward_scale_moments": (_I, [_P, _P, _P, _P, _P, _I, _I, _D, _P]),
    "dppo_reward_scale_apply": (_I, [_P, _P, _I, _I, _D, _D, _P]),
    "dppo_reward_scale_per_env": (_I, [_P, _P, _P, _P, _I, _P, _P, _I, _I, _D, _D, _D, _P, _P]),
    "dppo_reward_scale_per_env_moments": (_I, [_P, _P, _P, _P, _P, _I, _I, _D, _P]),
    "dppo_reward_scale_per_env_apply": (_I, [_P, _P, _I, _I, _I, _D, _D, _P, _P]),
    "dppo_gae": (_I, [_P, _P, _P, _P, _I, _I, _D, _D, _D, _P, _P, _P]),
    "dppo_ppo_workspace_bytes": (_SZ, [_DIMS, _I, _I]),
    "dppo_ppo_adv_stats": (_I, [_P, _I64, _I, _U64, _I, _I64, _I, _P, _P, _P]),
    "dppo_ppo_adv_stats_all": (_I, [_P, _I64, _I, _U64, _I, _I, _I64, _I, _P, _P]),
    "dppo_ppo_minibatch": (_I, [_DIMS, _I, ctypes.POINTER(DppoPpoHparams), _P, _P, _P, _P, _P, _P, _P, _P, _P,
                               _I64, _U64, _I, _I64, _I, _P, _P, _P, _P, _P, _P]),
    "dppo_pretrain_minibatch": (_I, [_DIMS, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I64, _F, _P, _P, _P, _P]),
    "dppo_ppo_minibatch_part": (_I, [_DIMS, _I, ctypes.POINTER(DppoPpoHparams), _P, _P, _P, _P, _P, _P, _P, _P,
                                    _P, _I64, _U64, _I, _I64, _I, _P, _P, _P, _P, _P, _I, _P]),
    "dppo_feistel_permute": (_I, [_I64, _I64, _I64, _U64, _I, _P, _P]),
    "dppo_adamw": (_I, [_P, _P, _P, _P, _I64, _I64, _F, _F, _F, _F, _F, _I, _P]),
    "dppo_copy_from_host": (_I, [_I, _P, _P, _P, _P]),
    "dppo_eta_step": (_I, [_P, _P, _I64, _F, _F, _F, _F, _F, _I, _F, _F, _P, _P, _I, _P, _P]),
    "dppo_pack_all": (_I, [_DIMS, _I, _P, _P, _P, _P, _P]),
    "dppo_optimizer_step": (_I, [_DIMS, _I, _P, _P, _P, _P, _I64, _I64, _F, _F, _F, _F, _F, _I, _P, _P, _P, _P, _P,
                                 _P, _I, _U64, _P]),
    "dppo_optimizer_step_ex": (_I, [_DIMS, _I, _P, _P, _P, _P, _I64, _I64, _F, _F, _F, _F, _F, _I, _P, _P, _P, _P,
                                    _P, _P, _I, _U64, _P, _P, _I, _P]),
    "dppo_ipc_region_bytes": (_SZ, [_I64]),
    "dppo_ipc_alloc": (_I, [_SZ, ctypes.POINTER(ctypes.c_void_p), _P]),
    "dppo_ipc_open": (_I, [_P, ctypes.POINTER(ctypes.c_void_p)]),
    "dppo_ipc_close": (_I, [_P]),
    "dppo_ipc_free": (_I, [_P]),
    "dppo_ipc_allreduce": (_I, [_P, _I, _I, _I64, _P, _I64, _U64, _P, _P]),
    "dppo_ppo_clear_ranges": (_I, [_DIMS, _I, _I, _P, _P, _I, _P, _P, ctypes.POINTER(ctypes.c_int)]),
    "dppo_value_moments": (_I, [_P, _P, _I64, _P, _P]),
    "dppo_episode_sums": (_I, [_P, _P, _I, _I, _I, _D, _P, _P]),
    "dppo_refresh_sampler_tables": (_I, [_P, _P]),
    "dppo_materialize_l2": (_I, [_DIMS, _I, _P, _P, _P, _I, _P]),
}

EXPORTED_SYMBOLS = tuple(_SIGNATURES)

_lib = None


ABI_VERSION = 15


class DppoError(RuntimeError):
    pass


def load(path=LIB_PATH):
    """Load and bind the library; raises if it is missing (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise DppoError(
            f"libdppo_hip.so not found at {path}. Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C diffusionpolicyoptimization_amd/csrc`. There is no CPU fallback.")
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dppo_abi_version() != ABI_VERSION:
        raise DppoError("libdppo_hip.so ABI version mismatch")
    _lib = lib
    return lib


def call(name, *args):
    lib = load()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise DppoError(f"{name} failed ({rc}): {lib.dppo_last_error().decode()}")
    return rc


def query(name, *args):
    return getattr(load(), name)(*args)


def ptr(t):
    """Device pointer of a torch tensor (None -> NULL)."""
    if t is None:
        return None
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
