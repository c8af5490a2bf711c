// dppo_internal.h — host-side helpers shared by the translation units of libdppo_hip.so.
#pragma once
#include <hip/hip_runtime.h>
#include "../../include/dppo.h"
#include "dppo_layout.h"

int dppo_set_error(int code, const char* fmt, ...);
int dppo_hip_fail(hipError_t e, const char* what);

int dppo_pack_mlp(int in_dim, int hidden, int out_dim, int time_dim, int precision, const float* params,
                  void* packed, hipStream_t s, int temb_steps = 0, int time_stride = 1);

// derived dimensions of a dppo_dims
struct Dims {
    int Do, Da, Ta, To, TD, H, HC, K, KF, TS;   // K = sampling steps, TS = time stride
    int XD, SD, IN;   // XD = Ta*Da, SD = To*Do, IN = XD + TD + SD
};
int dppo_check_dims(const dppo_dims* d, Dims* out);
// the images of the given networks (either may be null) and the actor's time tables, one launch;
// defer_sampler_tables: the actor's split-sampler tables are left stale and re-derived by the
// sampler before its next launch on that image (dppo_refresh_sampler_tables, pack.hip)
// zero_ptrs / zero_bytes: up to a few byte ranges (4-B aligned, sizes multiples of 4) the launch also zeroes
int dppo_pack_models(const Dims& D, int precision, const float* actor_params, void* packed_actor,
                     const float* critic_params, void* packed_critic, hipStream_t s, bool defer_sampler_tables = false,
                     void* const* zero_ptrs = nullptr, const size_t* zero_bytes = nullptr, int n_zero = 0);

// The pack of one network as per-element stores (DPPO_STEP_FUSED_PACK, update.hip): each job maps
// the elements [lo, hi) of the network's flat parameters to one image segment
struct FuseJob {
    int kind;          // 0 = packed [IK][IN] image from a row-major [IK][IN] tensor, 1 = packed [IK][IN]
                       // image of the transpose of a row-major [IN][IK] tensor, 2 = fp32 copy
    int IK, IN, KS;    // image rows / columns / k-steps
    int64_t lo, hi;
    uint8_t* dst;
};
constexpr int FUSE_MAXJ = 12;
// the jobs of the update-mode pack (PACK_UPDATE: no split-sampler tables) of one network whose flat
// parameters start at element 0 of the step's range; returns the job count (<= FUSE_MAXJ) or -1
int dppo_fuse_jobs(int in_dim, int hidden, int out_dim, int time_dim, int precision, void* packed, int temb_steps,
                   FuseJob* jobs);
// the row tiles' fold segments (RT_*) of an actor image, alone: after a fused actor step (pack.hip)
int dppo_pack_rt_fold(int in_dim, int hidden, int out_dim, int time_dim, int precision, const float* actor_params,
                      void* packed_actor, int temb_steps, int time_stride, hipStream_t s);
// temb: the TEMB table is stale too (the fused actor step), not only the split-sampler tables
int dppo_mark_tables_stale(const Dims& D, int precision, const float* actor_params, const void* packed_actor, bool temb);


// precision enum values the library implements; the two 2-byte operand policies share layouts
inline bool dppo_prec_ok(int p) { return p == DPPO_F32 || p == DPPO_BF16 || p == DPPO_F16; }
inline bool dppo_prec_2b(int p) { return p == DPPO_BF16 || p == DPPO_F16; }
// backward seed scale of a precision (PolicyF16::GRAD_SCALE): the row tiles seed the backward pass
// with this times the loss gradient; the weight-gradient outputs multiply by its inverse
inline float dppo_grad_scale(int p) { return p == DPPO_F16 ? 4096.f : 1.f; }
// the fp16 backward seed scale of a minibatch of global_rows rows: the largest power of two <=
// min(4096, global_rows). The seed is scale / global_rows x the per-row loss gradient, so it never
// exceeds the unscaled per-row gradient (a small minibatch with large value errors cannot overflow
// fp16), and at the bench's 50,000 rows it is the full 4096 that keeps the per-row gradients
// above fp16's subnormal range. A power of two: dividing it out of the fp32 dW is exact.
inline float dppo_grad_scale_rows(int p, int64_t global_rows) {
    if (p != DPPO_F16) return 1.f;
    float s = 1.f;
    while (s < 4096.f && (int64_t)(2.f * s) <= global_rows) s *= 2.f;
    return s;
}

#define DPPO_CHECK(cond, ...) do { if (!(cond)) return dppo_set_error(DPPO_EINVAL, __VA_ARGS__); } while (0)
#define DPPO_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return dppo_hip_fail(e_, #x); } while (0)

// ---- kernel timer (ABI 10, dppo_kernel_timing*): HIP events around the launches of the kernels
// below, on the launch's own stream, while enabled (one relaxed flag test per launch otherwise) ----
enum DppoKt {
    KT_SAMPLER, KT_ACTOR_TRAIN, KT_ACTOR_LOGPROB, KT_CRITIC_TRAIN, KT_CRITIC_FWD, KT_DW_ACTOR, KT_DW_CRITIC,
    KT_L2_BACK, KT_TIME_BWD, KT_ADAMW, KT_PACK_ALL, KT_GAE, KT_RETS, KT_MOMENTS, KT_SCALE_APPLY, KT_ZERO,
    KT_CRIT_ROWS, KT_ADV_STATS, KT_ALLREDUCE, KT_COUNT
};
extern volatile int g_dppo_kt_on;
int dppo_kt_begin(int id, hipStream_t s);   // -1 when disabled
void dppo_kt_end(int slot, hipStream_t s);
struct DppoKtScope {   // brackets the launches of one scope: { DppoKtScope kt(KT_GAE, s); launch; }
    int slot; hipStream_t s;
    DppoKtScope(int id, hipStream_t st) : slot(g_dppo_kt_on ? dppo_kt_begin(id, st) : -1), s(st) {}
    ~DppoKtScope() { if (slot >= 0) dppo_kt_end(slot, s); }
};

// the opt-in to `bytes` of dynamic LDS for kernel k: hipFuncSetAttribute only the first time k asks
// for that much (a host API call per launch otherwise)
int dppo_func_lds(const void* k, size_t bytes);
