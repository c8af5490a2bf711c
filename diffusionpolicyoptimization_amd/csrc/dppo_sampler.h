// dppo_sampler.h — launch arguments shared by the sampler kernels (sampler.hip: the weight-streaming
// kernel; sampler_split.hip: the register-resident split kernel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dppo_layout.h"

struct SampleArgs {
    const uint8_t* packed_base;
    const uint8_t* packed_ft;
    const float* sched;   // [K][8]
    const float* cond;    // [E][SD]
    const float* x_T;     // [E][XD] or null
    const float* noise;   // [K][E][XD] or null
    float* actions;       // [E][XD]
    float* chains;        // [E][KF+1][XD] or null
    float* cond_out;      // [E][SD] device copy of cond or null (cond may be mapped host memory)
    float* actions_host;  // [E][XD] mapped pinned host memory or null (zero-copy action hand-off)
    uint64_t* actions_tagged;  // [E][XD] tagged granules {cond_tag, fp32} in mapped host memory, or null
    // pre-enqueued rollout steps (dppo_rollout_*): wait until *go >= go_value before reading cond,
    // and add 1 to *done per workgroup after the actions are visible to the host (both counters
    // live in fine-grained host memory); null = an ordinary launch
    const uint32_t* go;
    uint32_t go_value;
    uint32_t* done;
    // tagged observation (dppo_rollout_enqueue_tagged): [E][SD] granules {tag << 32 | fp32 bits}
    // polled until every tag equals cond_tag (then cond is unused); null = cond / go as above
    const uint64_t* cond_tagged;
    uint32_t cond_tag;
    uint64_t seed;
    uint32_t call_id;
    int E, env_offset, deterministic;
    float min_std, randn_clip, final_clip;
    int XD, SD, TD, H, K, KF, IN;
    MlpLayout L;          // same layout for base and ft
};

// This workgroup's R (16 or 32) env rows of a TAGGED observation into st[R][SD]: every thread polls
// its granules (system-scope relaxed loads of mapped host memory) until each carries a.cond_tag — the
// value arrives with its own ready flag, so there is no separate flag round trip. Bounded (4 s):
// on timeout the step runs on what it read and (flag_timeout) sets bit 31 of *done.
template <int ST, int R = 16>
__device__ inline void sampler_load_state_tagged(const SampleArgs& a, int row0, float* st, bool flag_timeout, int tid) {
    const int SD = a.SD, n = R * SD;
    constexpr int NG = (R * 64 + ST - 1) / ST;      // SD <= 64 (dppo_check_dims)
    float v[NG];
    bool ok[NG];
#pragma unroll
    for (int u = 0; u < NG; ++u) {
        const int i = tid + u * ST;
        ok[u] = !(i < n && row0 + i / SD < a.E);
        v[u] = 0.f;
    }
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 400000000ull;   // 100 MHz: 4 s
    for (;;) {
        bool all = true;
#pragma unroll
        for (int u = 0; u < NG; ++u) {
            const int i = tid + u * ST;
            if (!ok[u]) {
                const uint64_t x = __hip_atomic_load(a.cond_tagged + (size_t)(row0 + i / SD) * SD + i % SD,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if ((uint32_t)(x >> 32) == a.cond_tag) {
                    ok[u] = true;
                    v[u] = __uint_as_float((uint32_t)x);
                }
            }
            all = all && ok[u];
        }
        if (__syncthreads_and(all)) break;
        if (__syncthreads_or(__builtin_amdgcn_s_memrealtime() > t_end)) {
            if (flag_timeout && tid == 0 && a.done)
                __hip_atomic_fetch_or(a.done, 0x80000000u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            break;
        }
        __builtin_amdgcn_s_sleep(2);
    }
#pragma unroll
    for (int u = 0; u < NG; ++u) {
        const int i = tid + u * ST;
        if (i < n) st[i] = v[u];
    }
}

// The split sampler (sampler_split.hip): returns DPPO_OK after launching, DPPO_EUNSUPPORTED (without
// touching the error message) when the shape is outside what it instantiates, or another error code.
int launch_sample_split(const SampleArgs& a, int precision, hipStream_t s);
// whether the split sampler takes this shape (same test launch_sample_split applies)
bool sample_split_supported(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF);
// workgroups (CUs) per 16-env group of the split sampler for this shape (4, or 8: the P = 8 kernel
// or the P = 4 kernel's two member sets), 0 = not taken
int split_members_for(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF);
int sampler_device_cus();   // CUs of the current device (0 if unknown)
// the split sampler's plan (dppo_sampler_plan): out[4] = kernel, members per set, sets, workgroups
void split_plan_query(int precision, int H, int XD, int SD, int ks_in, int E, int K, int KF, int* out);
