// api.hip — C-ABI plumbing of libdppo_hip.so: errors, dimension checks, sizes, packing entry points.
#include <stdarg.h>
#include <stdio.h>
#include <mutex>
#include <vector>
#include "dppo_common.cuh"
#include "dppo_internal.h"

static thread_local char g_err[512] = "";

int dppo_set_error(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int dppo_hip_fail(hipError_t e, const char* what) {
    return dppo_set_error(DPPO_EHIP, "HIP error %d (%s) in %s", (int)e, hipGetErrorString(e), what);
}

int dppo_check_dims(const dppo_dims* d, Dims* o) {
    DPPO_CHECK(d != nullptr, "dims is NULL");
    o->Do = d->obs_dim; o->Da = d->action_dim; o->Ta = d->horizon_steps; o->To = d->cond_steps;
    o->TD = d->time_dim; o->H = d->actor_hidden; o->HC = d->critic_hidden;
    o->K = d->denoising_steps; o->KF = d->ft_denoising_steps;
    o->TS = d->time_stride > 0 ? d->time_stride : 1;
    DPPO_CHECK(d->time_stride >= 0 && (int64_t)o->K * o->TS <= 1000, "time_stride out of range");
    DPPO_CHECK(o->Do > 0 && o->Da > 0 && o->Ta > 0 && o->To > 0, "obs/action/horizon/cond dims must be > 0");
    DPPO_CHECK(o->TD >= 4 && o->TD % 2 == 0 && o->TD <= 64, "time_dim must be even, in [4, 64]");
    DPPO_CHECK(o->H % 128 == 0 && o->H >= 128 && o->H <= 512, "actor_hidden must be 128/256/384/512");
    DPPO_CHECK(o->HC % 128 == 0 && o->HC >= 128 && o->HC <= 512, "critic_hidden must be 128/256/384/512");
    DPPO_CHECK(o->K >= 1 && o->K <= 1000, "denoising_steps out of range");
    DPPO_CHECK(o->KF >= 1 && o->KF <= o->K, "ft_denoising_steps must be in [1, denoising_steps]");
    o->XD = o->Ta * o->Da;
    o->SD = o->To * o->Do;
    o->IN = o->XD + o->TD + o->SD;
    DPPO_CHECK(o->XD <= 32, "horizon_steps*action_dim must be <= 32");
    DPPO_CHECK(o->SD <= 64, "cond_steps*obs_dim must be <= 64");
    return DPPO_OK;
}

extern "C" int dppo_abi_version(void) { return DPPO_ABI_VERSION; }
extern "C" const char* dppo_last_error(void) { return g_err; }

extern "C" size_t dppo_actor_param_count(const dppo_dims* d) {
    Dims D;
    if (dppo_check_dims(d, &D)) return 0;
    return make_flat_offsets(D.IN, D.H, D.XD, D.TD).count;
}
extern "C" size_t dppo_critic_param_count(const dppo_dims* d) {
    Dims D;
    if (dppo_check_dims(d, &D)) return 0;
    return make_flat_offsets(D.SD, D.HC, 1, 0).count;
}
extern "C" size_t dppo_actor_packed_bytes(const dppo_dims* d, int precision) {
    Dims D;
    if (dppo_check_dims(d, &D)) return 0;
    return make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K).total;
}
extern "C" size_t dppo_critic_packed_bytes(const dppo_dims* d, int precision) {
    Dims D;
    if (dppo_check_dims(d, &D)) return 0;
    return make_mlp_layout(D.SD, D.HC, 1, 0, precision).total;
}
extern "C" int dppo_pack_actor(const dppo_dims* d, int precision, const float* params, void* packed, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(params && packed, "dppo_pack_actor: null pointer");
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    return dppo_pack_mlp(D.IN, D.H, D.XD, D.TD, precision, params, packed, (hipStream_t)stream, D.K, D.TS);
}
extern "C" int dppo_pack_critic(const dppo_dims* d, int precision, const float* params, void* packed, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(params && packed, "dppo_pack_critic: null pointer");
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    return dppo_pack_mlp(D.SD, D.HC, 1, 0, precision, params, packed, (hipStream_t)stream);
}

// ---- kernel timer: (start, end) event pairs per launch of a timed kernel, summed on read ----
volatile int g_dppo_kt_on = 0;
namespace {
const char* const kKtNames[KT_COUNT] = {
    "sampler", "actor_rowtile_train", "actor_rowtile_logprob", "critic_rowtile_train",
    "critic_rowtile_forward", "dw_kernel_actor", "dw_kernel_critic", "l2_back_kernel", "time_bwd_kernel",
    "adamw_kernel", "pack_all_kernel", "gae_kernel", "rets_kernel", "moments_kernel", "scale_apply_kernel",
    "zero_kernel", "crit_rows_kernel", "adv_stats_kernel", "ipc_allreduce_kernel"};
struct KtRec { int id; hipEvent_t e0, e1; };
std::mutex g_kt_mu;
std::vector<KtRec> g_kt;     // event pool; [0, g_kt_used) hold this window's launches
size_t g_kt_used = 0;
}

int dppo_kt_begin(int id, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_kt_mu);
    if (!g_dppo_kt_on || id < 0 || id >= KT_COUNT) return -1;
    if (g_kt_used == g_kt.size()) {
        KtRec r{id, nullptr, nullptr};
        if (hipEventCreate(&r.e0) != hipSuccess || hipEventCreate(&r.e1) != hipSuccess) {
            (void)hipGetLastError();
            return -1;
        }
        g_kt.push_back(r);
    }
    KtRec& r = g_kt[g_kt_used];
    r.id = id;
    if (hipEventRecord(r.e0, s) != hipSuccess) { (void)hipGetLastError(); return -1; }
    return (int)g_kt_used++;
}

void dppo_kt_end(int slot, hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_kt_mu);
    if (slot >= 0 && (size_t)slot < g_kt_used && hipEventRecord(g_kt[slot].e1, s) != hipSuccess) (void)hipGetLastError();
}

extern "C" int dppo_kernel_timing(int enable) {
    std::lock_guard<std::mutex> lk(g_kt_mu);
    g_dppo_kt_on = enable ? 1 : 0;
    g_kt_used = 0;
    return DPPO_OK;
}

extern "C" const char* dppo_kernel_timing_name(int id) { return id >= 0 && id < KT_COUNT ? kKtNames[id] : nullptr; }

extern "C" int dppo_kernel_timing_read(int n, double* total_ms, int64_t* launches) {
    DPPO_CHECK(n >= 0 && (n == 0 || (total_ms && launches)), "dppo_kernel_timing_read: bad arguments");
    std::lock_guard<std::mutex> lk(g_kt_mu);
    for (int i = 0; i < n; ++i) { total_ms[i] = 0.0; launches[i] = 0; }
    for (size_t k = 0; k < g_kt_used; ++k) {
        const KtRec& r = g_kt[k];
        DPPO_HIP(hipEventSynchronize(r.e1));
        float ms = 0.f;
        DPPO_HIP(hipEventElapsedTime(&ms, r.e0, r.e1));
        if (r.id < n) { total_ms[r.id] += ms; launches[r.id] += 1; }
    }
    g_kt_used = 0;
    return DPPO_OK;
}

namespace {
std::mutex g_lds_mu;
std::vector<std::pair<const void*, size_t>> g_lds;
}
int dppo_func_lds(const void* k, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_lds_mu);
    for (auto& e : g_lds)
        if (e.first == k) {
            if (bytes <= e.second) return DPPO_OK;
            DPPO_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
            e.second = bytes;
            return DPPO_OK;
        }
    DPPO_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    g_lds.emplace_back(k, bytes);
    return DPPO_OK;
}
