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
    // pre-enqueued rollout steps (dppo_rollout_*): wait until *go >= go_value before reading cond,
    // and add 1 to *done per workgroup after the actions are visible to the host (both counters
    // live in fine-grained host memory); null = an ordinary launch
    const uint32_t* go;
    uint32_t go_value;
    uint32_t* done;
    uint64_t seed;
    uint32_t call_id;
    int E, env_offset, deterministic;
    float min_std, randn_clip, final_clip;
    int XD, SD, TD, H, K, KF, IN;
    MlpLayout L;          // same layout for base and ft
};

// The split sampler (sampler_split.hip): returns DPPO_OK after launching, DPPO_EUNSUPPORTED (without
// touching the error message) when the shape is outside what it instantiates, or another error code.
int launch_sample_split(const SampleArgs& a, int precision, hipStream_t s);
// whether the split sampler takes this shape (same test launch_sample_split applies)
bool sample_split_supported(int precision, int H, int XD, int ks_in, int E, int K);
// workgroups (CUs) per 16-env group of the split sampler
int split_sampler_members();
