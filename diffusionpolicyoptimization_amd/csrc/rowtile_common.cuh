// rowtile_common.cuh — pieces shared by the row-tile kernels (rowtile.hip, rowtile128.hip): the
// permuted feature-major image layout, accumulator stores, bias add, metric atomics.
#pragma once
#include "dppo_ppo.h"

#define LOG_2PI_HALF 0.91893853320467274178f

// Feature-major images XT[col][row] hold the rows of each 16*MT-row tile in a PERMUTED order:
// position p of a tile holds row img_row(p), so that the 8 rows one lane holds for a column across
// an (even, odd) pair of MFMA tiles (rows 16m + 4j + 0..3 of tiles m = 2P, 2P+1, j = lane >> 4) are
// 8 consecutive positions and leave as ONE 16-byte store (8-byte per-lane stores made the image
// writes store-issue bound). Every image of a dW pair and the actor's seg[] use the same order;
// the dW GEMM sums over rows, so the order is invisible in its result.
__device__ inline int img_pos(int r) {
    const int m = r >> 4;
    return 32 * (m >> 1) + 8 * ((r >> 2) & 3) + 4 * (m & 1) + (r & 3);
}
__device__ inline int img_row(int p) {
    return 16 * (2 * (p >> 5) + ((p >> 2) & 1)) + 4 * ((p >> 3) & 3) + (p & 3);
}

// Accumulator tile -> feature-major image. Buffer stores through ONE resource for the whole
// workspace: the per-lane part of the offset is a single 32-bit VGPR, the image / tile parts are
// scalar, so no 64-bit address pairs are kept live across the unrolled layers.
template <class P, int MT, int NT>
__device__ inline void store_accT(__amdgpu_buffer_rsrc_t ws, uint32_t img_off, uint32_t ldm, int ntile0, uint32_t grow0,
                                  int lane, const f32x4 (&v)[MT][NT]) {
    static_assert(MT % 2 == 0, "image rows are permuted over MFMA tile pairs");
    using AT = typename P::AT;
    constexpr uint32_t es = sizeof(AT);
    const uint32_t vo = ((uint32_t)ccol(lane) * ldm + (uint32_t)((lane >> 4) << 3)) * es;
    const uint32_t so0 = img_off + ((uint32_t)ntile0 * 16u * ldm + grow0) * es;
#pragma unroll
    for (int mp = 0; mp < MT / 2; ++mp)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const uint32_t so = so0 + ((uint32_t)n * 16u * ldm + (uint32_t)mp * 32u) * es;
            const f32x4 lo = v[2 * mp][n], hi = v[2 * mp + 1][n];
            if constexpr (es == 2) {
                const u32x4 e = {P::pack2(lo[0], lo[1]), P::pack2(lo[2], lo[3]),
                                 P::pack2(hi[0], hi[1]), P::pack2(hi[2], hi[3])};
                // soffset must be the literal 0: with an SGPR there, hipcc (ROCm 7.2) does not guard
                // the >8-byte store-data hazard (a following VALU overwrote the 4th dword)
                __builtin_amdgcn_raw_buffer_store_b128(e, ws, vo + so, 0, 0);
            } else {
                // 8-B stores: the 16-B buffer_store form came out with a corrupted 4th dword under
                // hipcc 7.2 for gfx950 in the fp32 critic (a store-data hazard the compiler does
                // not guard); fp32 is the parity mode, so exactness wins here
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(lo[0]), __float_as_uint(lo[1])}, ws, vo, so, 0);
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(lo[2]), __float_as_uint(lo[3])}, ws, vo, so + 8, 0);
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(hi[0]), __float_as_uint(hi[1])}, ws, vo, so + 16, 0);
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(hi[2]), __float_as_uint(hi[3])}, ws, vo, so + 24, 0);
            }
        }
}

// image positions [8g, 8g + 8) of column c (rows img_row(p), value(r)) in one 16-B store (bf16)
// or four 8-B stores (fp32)
template <class P, class F>
__device__ inline void store_img8(void* img, size_t ldm, size_t grow0, int c, int g, F value) {
    using AT = typename P::AT;
    float e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = value(img_row(8 * g + k));
    AT* dst = (AT*)img + (size_t)c * ldm + grow0 + 8 * g;
    if constexpr (sizeof(AT) == 2) {
        *(u32x4*)dst = u32x4{P::pack2(e[0], e[1]), P::pack2(e[2], e[3]),
                             P::pack2(e[4], e[5]), P::pack2(e[6], e[7])};
    } else {
#pragma unroll
        for (int k = 0; k < 8; k += 2) *(u32x2*)(dst + k) = u32x2{__float_as_uint(e[k]), __float_as_uint(e[k + 1])};
    }
}

template <class P, int MT, int NT>
__device__ inline void store_acc_lds(typename P::AT* T, int ld, int ntile0, int lane, const f32x4 (&v)[MT][NT]) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const int col = (ntile0 + n) * 16 + ccol(lane);
#pragma unroll
            for (int r = 0; r < 4; ++r) T[(m * 16 + crow(lane, r)) * ld + col] = P::cvt(v[m][n][r]);
        }
}

template <int MT, int NT>
__device__ inline void add_bias(f32x4 (&v)[MT][NT], const float* __restrict__ b, int ntile0, int lane) {
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        const float bv = b[(ntile0 + n) * 16 + ccol(lane)];
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[m][n][r] += bv;
    }
}

__device__ inline void atomic_add_metric(double* m, int i, double v) { atomicAdd(m + i, v); }

