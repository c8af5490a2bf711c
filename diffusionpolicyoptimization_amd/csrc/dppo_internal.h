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

#define DPPO_CHECK(cond, ...) do { if (!(cond)) return dppo_set_error(DPPO_EINVAL, __VA_ARGS__); } while (0)
#define DPPO_HIP(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) return dppo_hip_fail(e_, #x); } while (0)
