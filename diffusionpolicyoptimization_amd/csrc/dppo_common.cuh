// dppo_common.cuh — shared device code for the gfx950 DPPO kernels.
//
// Design: every MLP layer is an MFMA GEMM whose A operand (activations)
// sits in LDS as a row-major tile and whose B operand (weights) is streamed from global memory
// (L2/MALL resident) in a PRE-PACKED fragment order, so each wave-instruction of the weight
// stream is one fully-coalesced 1 KiB `global_load_dwordx4`. Two precision policies share the
// code: bf16 (v_mfma_f32_16x16x32_bf16) and fp32 (v_mfma_f32_16x16x4_f32, exact fp32 products,
// used for parity). Both consume 16 bytes of A and 16 bytes of B per lane per "k-step".
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "dppo_layout.h"

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) float f32x2_t;

typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;

// two floats -> packed bf16 pair (RNE) in ONE v_cvt_pk_bf16_f32; two scalar (__bf16) casts
// compile to two conversions plus a shift and an or
__device__ inline unsigned int dppo_pack_bf16x2(float lo, float hi) {
    return __builtin_bit_cast(unsigned int, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}
// two floats -> packed fp16 pair (RNE, v_cvt_pk_f16_f32)
__device__ inline unsigned int dppo_pack_f16x2(float lo, float hi) {
    return __builtin_bit_cast(unsigned int, __builtin_convertvector((f32x2_t){lo, hi}, f16x2_t));
}

// One DDPM posterior step of the samplers (diffusion.py:198-201 x0 reconstruction + clip at 1,
// :239-242 posterior mean, diffusion_vpg.py:301-320 mean + std z) with every product and sum rounded
// on its own, as NumPy / TF evaluate it: no FMA contraction, so every sampler path (split, XR, pair,
// P = 8, streaming) gives the same bits whatever the compiler does around it.
__device__ inline float ddpm_post(float c0, float c1, float c2, float c3, float sd, float x, float ep, float z) {
#pragma clang fp contract(off)
    float x0 = c0 * x - c1 * ep;
    x0 = fminf(fmaxf(x0, -1.f), 1.f);
    const float mu = c2 * x0 + c3 * x;
    return mu + sd * z;
}

#define DPPO_WAVES 8
#define DPPO_THREADS (DPPO_WAVES * 64)

// ------------------------------------------------------------------------------------------------
// precision policies
// ------------------------------------------------------------------------------------------------
struct PolicyBF16 {
    using AT = __bf16;                 // activation element type in LDS
    static constexpr int KG = 32;      // k covered by one 16-B fragment
    static constexpr int EPL = 8;      // elements per lane per fragment
    static constexpr float GRAD_SCALE = 1.f;   // backward seed scale (range of the 2-byte images)
    __device__ static inline AT cvt(float x) { return (__bf16)x; }
    __device__ static inline float tof(AT x) { return (float)x; }
    __device__ static inline unsigned int pack2(float lo, float hi) { return dppo_pack_bf16x2(lo, hi); }
    // the two halves of a packed pair back to fp32
    __device__ static inline float lo2f(unsigned int w) { return __uint_as_float(w << 16); }
    __device__ static inline float hi2f(unsigned int w) { return __uint_as_float(w & 0xffff0000u); }
    __device__ static inline f32x4 mma(u32x4 a, u32x4 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                       __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
    }
};

// fp16 operands (BASELINE config 5): v_mfma_f32_16x16x32_f16, same fragment geometry as bf16.
// fp16's 5-bit exponent does not hold the PPO gradients (~1e-5 per row at b = 50,000), so the
// backward pass is seeded with GRAD_SCALE times the loss gradient and the weight-gradient outputs
// (fp32) are multiplied by 1 / GRAD_SCALE (a power of two: exact).
struct PolicyF16 {
    using AT = _Float16;
    static constexpr int KG = 32;
    static constexpr int EPL = 8;
    static constexpr float GRAD_SCALE = 4096.f;
    __device__ static inline AT cvt(float x) { return (_Float16)x; }
    __device__ static inline float tof(AT x) { return (float)x; }
    __device__ static inline unsigned int pack2(float lo, float hi) { return dppo_pack_f16x2(lo, hi); }
    __device__ static inline float lo2f(unsigned int w) {
        return (float)__builtin_bit_cast(_Float16, (unsigned short)(w & 0xffffu));
    }
    __device__ static inline float hi2f(unsigned int w) {
        return (float)__builtin_bit_cast(_Float16, (unsigned short)(w >> 16));
    }
    __device__ static inline f32x4 mma(u32x4 a, u32x4 b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                      __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
    }
};

struct PolicyF32 {
    using AT = float;
    static constexpr int KG = 16;
    static constexpr int EPL = 4;
    static constexpr float GRAD_SCALE = 1.f;
    __device__ static inline AT cvt(float x) { return x; }
    __device__ static inline float tof(AT x) { return x; }
    // lane holds k = 4*(lane>>4) + q of the 16-k group for q = 0..3; MFMA q pairs A and B
    // entries of the same k, so the four 16x16x4 products sum the whole group.
    // NOTE: bit-cast the whole vector, then index. Per-component __builtin_bit_cast(float, a.y)
    // is miscompiled by hipcc (ROCm 7.2): all four MFMAs received component x.
    __device__ static inline f32x4 mma(u32x4 a, u32x4 b, f32x4 c) {
        const f32x4 af = __builtin_bit_cast(f32x4, a);
        const f32x4 bf = __builtin_bit_cast(f32x4, b);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(af[0], bf[0], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(af[1], bf[1], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(af[2], bf[2], c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_16x16x4f32(af[3], bf[3], c, 0, 0, 0);
        return c;
    }
};

template <class P> __device__ __host__ constexpr int lds_pad_elems() { return 32 / (int)sizeof(typename P::AT); }

// ------------------------------------------------------------------------------------------------
// fragment access
// ------------------------------------------------------------------------------------------------
// A fragment: row (lane & 15) of row-tile mt, k-step ks; 16 contiguous bytes in LDS.
template <class P>
__device__ inline u32x4 lds_afrag(const typename P::AT* A, int lda, int mt, int ks, int lane) {
    const typename P::AT* p = A + (mt * 16 + (lane & 15)) * lda + ks * P::KG + (lane >> 4) * P::EPL;
    return *reinterpret_cast<const u32x4*>(p);
}

// B fragments come from a packed image through a buffer resource (SGPRs): the per-load offset
// ((ntile*KS + ks) * 1 KiB + segment offset) is wave-uniform scalar arithmetic and the lane part
// is one constant VGPR, so the fully unrolled weight stream holds no 64-bit VGPR addresses.
struct WSrc {
    __amdgpu_buffer_rsrc_t rsrc;   // the whole packed image
    uint32_t off;                  // byte offset of this packed matrix in the image
};
__device__ inline __amdgpu_buffer_rsrc_t packed_rsrc(const void* image) {
    // raw buffer (stride 0), range 2 GiB, gfx9-family dword3 (DATA_FORMAT = 32)
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(image), (short)0, 0x7FFFFFFF, 0x00020000);
}
__device__ inline WSrc wsrc(__amdgpu_buffer_rsrc_t r, size_t off) { return WSrc{r, (uint32_t)off}; }
__device__ inline u32x4 load_bfrag_c(WSrc W, int KS, int ntile, int ks, int lane) {
    const uint32_t so = W.off + ((uint32_t)(ntile * KS + ks) << 10);
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(W.rsrc, lane << 4, so, 0));
}
// wave index as a scalar (threadIdx-derived values are VGPRs unless the compiler is told)
__device__ inline int wave_id() { return __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)); }

__device__ inline void zero_acc(f32x4& a) { a = f32x4{0.f, 0.f, 0.f, 0.f}; }

// ------------------------------------------------------------------------------------------------
// The weight stream. Each wave walks its fragments of every layer as one continuous stream: a
// register ring holds the next TWO k-steps (NT fragments each), and the tail of a layer already
// loads the first two k-steps of the NEXT layer, so the load queue never drains at a layer
// boundary. Every packed matrix has an even k-step count (dppo_layout.h), so the loop body is
// branch-free (the source switch is a scalar select) and hipcc emits counted vmcnt waits.
// ------------------------------------------------------------------------------------------------
template <int NT>
struct WRing {
    u32x4 b0[NT], b1[NT];
};

struct NextLayer {
    WSrc W;           // packed matrix the stream continues into (may repeat the current one)
    int KS, ntile0;
};

template <int NT>
__device__ inline void ring_prime(WRing<NT>& R, WSrc W, int KS, int ntile0, int lane) {
#pragma unroll
    for (int n = 0; n < NT; ++n) {
        R.b0[n] = load_bfrag_c(W, KS, ntile0 + n, 0, lane);
        R.b1[n] = load_bfrag_c(W, KS, ntile0 + n, 1, lane);
    }
}

// acc[MT][NT] = A[16*MT rows][KS*KG] x W[:, ntile0*16 .. (ntile0+NT)*16)   (W from the ring).
// KS is a template parameter: the layer is straight-line code, so the waitcnt pass emits exact
// counted vmcnt waits (a runtime trip count lets hipcc rotate the ring across the back-edge and
// fall back to vmcnt(0) every k-step).
template <class P, int MT, int NT, int KS>
__device__ inline void gemm_stream(const typename P::AT* A, int lda, WSrc W, int ntile0,
                                   f32x4 (&acc)[MT][NT], int lane, WRing<NT>& R, NextLayer nx) {
    static_assert(KS % 2 == 0, "packed k-step counts are even");
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NT; ++n) zero_acc(acc[m][n]);
#pragma unroll
    for (int ks = 0; ks < KS; ks += 2) {
        const bool in = ks + 2 < KS;
        const WSrc src = in ? W : nx.W;
        const int kss = in ? KS : nx.KS;
        const int nt0 = in ? ntile0 : nx.ntile0;
        const int k0 = in ? ks + 2 : 0;
        u32x4 c[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) c[n] = R.b0[n];
#pragma unroll
        for (int n = 0; n < NT; ++n) R.b0[n] = load_bfrag_c(src, kss, nt0 + n, k0, lane);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const u32x4 a = lds_afrag<P>(A, lda, m, ks, lane);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = P::mma(a, c[n], acc[m][n]);
        }
#pragma unroll
        for (int n = 0; n < NT; ++n) c[n] = R.b1[n];
#pragma unroll
        for (int n = 0; n < NT; ++n) R.b1[n] = load_bfrag_c(src, kss, nt0 + n, k0 + 1, lane);
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const u32x4 a = lds_afrag<P>(A, lda, m, ks + 1, lane);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = P::mma(a, c[n], acc[m][n]);
        }
    }
}

// Deeper weight stream for the latency-bound sampler: a D-deep queue of k-steps per wave (D*NT
// fragments in flight). In fully unrolled code the shifts are register renames; across the
// runtime denoising loop the queue is loop-carried with the next k-step always in slot 0. The
// look-ahead may run D k-steps past the end of a layer, through up to two following layers.
template <int D, int NT>
struct WQueue {
    u32x4 b[D][NT];
};

struct NextLayers {
    WSrc W1; int KS1;   // the layer after the current one
    WSrc W2; int KS2;   // and the one after that (for look-ahead past a short layer)
};

// fragment j of the stream that is at layer W (KS k-steps) and continues into nx.W1, nx.W2
template <int KS>
__device__ inline u32x4 stream_frag(WSrc W, const NextLayers& nx, int ntile, int j, int lane) {
    if (j < KS) return load_bfrag_c(W, KS, ntile, j, lane);                  // compile-time branch
    const int j1 = j - KS;
    const bool first = j1 < nx.KS1;                                           // wave-uniform
    const WSrc src = first ? nx.W1 : nx.W2;
    return load_bfrag_c(src, first ? nx.KS1 : nx.KS2, ntile, first ? j1 : j1 - nx.KS1, lane);
}

template <int D, int NT>
__device__ inline void queue_prime(WQueue<D, NT>& Q, WSrc W, int KS, const NextLayers& nx, int ntile0, int lane) {
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
        for (int n = 0; n < NT; ++n) {
            const bool in = d < KS;
            const int j1 = d - KS;
            const bool first = j1 < nx.KS1;
            Q.b[d][n] = in ? load_bfrag_c(W, KS, ntile0 + n, d, lane)
                           : load_bfrag_c(first ? nx.W1 : nx.W2, first ? nx.KS1 : nx.KS2, ntile0 + n,
                                          first ? j1 : j1 - nx.KS1, lane);
        }
}

// ZERO = false accumulates onto acc (a GEMM over a concatenated K); TAIL = true issues no
// look-ahead past this layer (the last layer of the kernel: nothing would consume it)
template <class P, int MT, int NT, int KS, int D, bool ZERO = true, bool TAIL = false>
__device__ inline void gemm_queue(const typename P::AT* A, int lda, WSrc W, int ntile0, f32x4 (&acc)[MT][NT], int lane,
                                  WQueue<D, NT>& Q, const NextLayers& nx) {
    if constexpr (ZERO) {
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int n = 0; n < NT; ++n) zero_acc(acc[m][n]);
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
        u32x4 c[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) c[n] = Q.b[0][n];
#pragma unroll
        for (int d = 0; d + 1 < D; ++d)
#pragma unroll
            for (int n = 0; n < NT; ++n) Q.b[d][n] = Q.b[d + 1][n];
        if (!TAIL || ks + D < KS) {
#pragma unroll
            for (int n = 0; n < NT; ++n) Q.b[D - 1][n] = stream_frag<KS>(W, nx, ntile0 + n, ks + D, lane);
        }
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const u32x4 a = lds_afrag<P>(A, lda, m, ks, lane);
#pragma unroll
            for (int n = 0; n < NT; ++n) acc[m][n] = P::mma(a, c[n], acc[m][n]);
        }
    }
}

// hidden-layer k-steps for a precision and n-tiles-per-wave (H = 16*NT*WAVES)
template <class P> __host__ __device__ constexpr int ksh_for(int NT, int WAVES = DPPO_WAVES) { return NT * 16 * WAVES / P::KG; }

// Narrow layer (out-Dense, n-tiles < waves): k-steps dealt round-robin over the 8 waves, NOK per
// wave (host guarantees KS == 8*NOK). The fragments are fetched early (out_prefetch, issued a
// layer or more ahead) so the narrow layer itself waits on nothing; partials reduce through LDS.
template <int NOK, int NO>
struct ORing {
    u32x4 b[NOK][NO];
};

template <int NOK, int NO, int WAVES = DPPO_WAVES>
__device__ inline void out_prefetch(ORing<NOK, NO>& O, WSrc W, int KS, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < NOK; ++i)
#pragma unroll
        for (int n = 0; n < NO; ++n) O.b[i][n] = load_bfrag_c(W, KS, n, wave + WAVES * i, lane);
}

template <class P, int MT, int NOK, int NO, int WAVES = DPPO_WAVES>
__device__ inline void gemm_narrow_pre(const typename P::AT* A, int lda, const ORing<NOK, NO>& O,
                                       f32x4 (&acc)[MT][NO], int wave, int lane) {
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int n = 0; n < NO; ++n) zero_acc(acc[m][n]);
#pragma unroll
    for (int i = 0; i < NOK; ++i)
#pragma unroll
        for (int m = 0; m < MT; ++m) {
            const u32x4 a = lds_afrag<P>(A, lda, m, wave + WAVES * i, lane);
#pragma unroll
            for (int n = 0; n < NO; ++n) acc[m][n] = P::mma(a, O.b[i][n], acc[m][n]);
        }
}

// out-layer k-steps per wave when H = 16*NT*WAVES (KS_h = H / KG dealt over WAVES waves)
template <class P> __host__ __device__ constexpr int nok_for(int NT) { return NT * 16 / P::KG; }

// Workgroup barrier for LDS hand-offs that leaves global loads in flight: waits for this wave's
// LDS ops only (a __syncthreads() would also emit s_waitcnt vmcnt(0) and drain the weight stream).
// The empty asm statements stop the compiler moving memory operations across the barrier.
__device__ inline void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// C/D fragment coordinates (dtype independent on gfx950): col = lane&15, row = 4*(lane>>4) + r
__device__ inline int crow(int lane, int r) { return ((lane >> 4) << 2) + r; }
__device__ inline int ccol(int lane) { return lane & 15; }

// ------------------------------------------------------------------------------------------------
// activations (Keras: relu, mish = x * tanh(softplus(x)))
// ------------------------------------------------------------------------------------------------
// mish(x) = x tanh(softplus(x)) = x n/(n+2) with n = e^x (e^x + 2): one v_exp + one v_rcp instead of
// the libm log1p/tanh routines (which inline to hundreds of instructions each and blow the
// instruction cache of the critic kernels). Relative error <= 2e-6 vs the exact form (checked
// against float64 over [-30, 30]); x > 15 is mish = x, mish' = 1 to fp32 precision.
__device__ inline float mishf(float x) {
    const float e = __expf(fminf(x, 15.f));
    const float n = e * (e + 2.f);
    return x > 15.f ? x : x * n * __builtin_amdgcn_rcpf(n + 2.f);
}
__device__ inline float mish_gradf(float x) {
    // opaque copy: stops hipcc from sharing e/n with a forward mishf of the same value, which
    // would keep them live from the forward to the backward pass (register spills)
    asm volatile("" : "+v"(x));
    const float e = __expf(fminf(x, 15.f));
    const float n = e * (e + 2.f);
    const float r = __builtin_amdgcn_rcpf(n + 2.f);
    return x > 15.f ? 1.f : n * r + 4.f * x * e * (e + 1.f) * r * r;
}

// ------------------------------------------------------------------------------------------------
// t_emb(t) = Dense(2TD->TD)(mish(Dense(TD->2TD)(SinusoidalPosEmb(t)))) (mlp_diffusion.py:40-45,
// modules.py:4-15), element by element. p: the actor's flat parameters (time_w1 [TD][2TD], time_b1,
// time_w2 [2TD][TD], time_b2 at the given offsets). The dot products are explicit fmaf chains: the
// pack's per-row blocks (pack.hip) and the fused optimizer step's last workgroup (update.hip) then
// agree bit for bit whatever the compiler contracts in each kernel (left to it, the same source
// compiled to different contractions in the two: last-ulp differences).
// ------------------------------------------------------------------------------------------------
__device__ inline float temb_sinusoid(int j, int t, int TD) {
    const int half = TD / 2;
    const float lnf = logf(10000.f) / (float)(half - 1);
    const float f = expf(-(float)(j % half) * lnf) * (float)t;
    return j < half ? sinf(f) : cosf(f);
}
__device__ inline float temb_hidden(const float* p, size_t w1, size_t b1, const float* te, int TD, int h) {
    float acc = p[b1 + h];
#pragma unroll 16
    for (int k = 0; k < TD; ++k) acc = __builtin_fmaf(te[k], p[w1 + (size_t)k * 2 * TD + h], acc);
    return mishf(acc);
}
__device__ inline float temb_output(const float* p, size_t w2, size_t b2, const float* a1, int TD, int j) {
    float acc = p[b2 + j];
#pragma unroll 16
    for (int k = 0; k < 2 * TD; ++k) acc = __builtin_fmaf(a1[k], p[w2 + (size_t)k * TD + j], acc);
    return acc;
}
// The R rows of the TEMB table (row r = t_emb(r TS)) by one workgroup; sm: 3 R TD floats of LDS
__device__ inline void temb_rows_block(const float* p, int64_t w1, int64_t b1, int64_t w2,
                                                                  int64_t b2, int TD, int TS, int R, float* out,
                                                                  float* sm) {
    const int tid = (int)threadIdx.x, nt = (int)blockDim.x;
    float* te = sm;              // [R][TD]
    float* a1 = sm + R * TD;     // [R][2TD]
    for (int i = tid; i < R * TD; i += nt) te[i] = temb_sinusoid(i % TD, (i / TD) * TS, TD);
    __syncthreads();
    for (int i = tid; i < R * 2 * TD; i += nt) a1[i] = temb_hidden(p, w1, b1, te + (i / (2 * TD)) * TD, TD, i % (2 * TD));
    __syncthreads();
    for (int i = tid; i < R * TD; i += nt) out[i] = temb_output(p, w2, b2, a1 + (i / TD) * 2 * TD, TD, i % TD);
}

// ------------------------------------------------------------------------------------------------
// Philox4x32-10 + Box-Muller (restated bit-for-bit by oracle/philox.py)
// ------------------------------------------------------------------------------------------------
struct u32x4s { uint32_t x, y, z, w; };
__device__ __host__ inline u32x4s philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                               uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    return u32x4s{c0, c1, c2, c3};
}
__device__ inline float u32_unit(uint32_t w) { return ((float)(w >> 9) + 0.5f) * (1.0f / 8388608.0f); }

// normal #q (0..3) of the Philox block (group, row, slot, call)
__device__ inline float philox_normal(uint64_t seed, uint32_t group, uint32_t row, uint32_t slot,
                                      uint32_t call, int q) {
    const u32x4s w = philox4x32_10(group, row, slot, call, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float ua = u32_unit(q < 2 ? w.x : w.z);
    const float ub = u32_unit(q < 2 ? w.y : w.w);
    const float r = sqrtf(-2.0f * logf(ua));
    const float ang = 6.283185307179586f * ub;
    return (q & 1) ? r * sinf(ang) : r * cosf(ang);
}

// all 4 normals of the block: the same values philox_normal gives for q = 0..3
__device__ inline void philox_normal4(uint64_t seed, uint32_t group, uint32_t row, uint32_t slot, uint32_t call,
                                      float (&z)[4]) {
    const u32x4s w = philox4x32_10(group, row, slot, call, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float r0 = sqrtf(-2.0f * logf(u32_unit(w.x))), a0 = 6.283185307179586f * u32_unit(w.y);
    const float r1 = sqrtf(-2.0f * logf(u32_unit(w.z))), a1 = 6.283185307179586f * u32_unit(w.w);
    z[0] = r0 * cosf(a0); z[1] = r0 * sinf(a0);
    z[2] = r1 * cosf(a1); z[3] = r1 * sinf(a1);
}

// ------------------------------------------------------------------------------------------------
// Feistel minibatch permutation (restated by oracle/philox.py:feistel_permute)
// ------------------------------------------------------------------------------------------------
struct FeistelKey { uint32_t k[4]; int half_bits; uint64_t n; };
__host__ __device__ inline FeistelKey feistel_key(uint64_t n, uint64_t seed, int epoch) {
    FeistelKey f;
    int hb = 1;
    while ((1ull << (2 * hb)) < n) ++hb;
    f.half_bits = hb;
    f.n = n;
    const u32x4s w = philox4x32_10((uint32_t)epoch, 0x5EEDu, 0u, 0u, (uint32_t)seed, (uint32_t)(seed >> 32));
    f.k[0] = w.x; f.k[1] = w.y; f.k[2] = w.z; f.k[3] = w.w;
    return f;
}
__host__ __device__ inline uint64_t feistel_once(uint64_t x, const FeistelKey& f) {
    const uint64_t mask = (1ull << f.half_bits) - 1;
    uint64_t l = (x >> f.half_bits) & mask, r = x & mask;
    for (int i = 0; i < 4; ++i) {
        uint32_t h = (uint32_t)(r ^ f.k[i]);
        h *= 0x9E3779B1u; h ^= h >> 15; h *= 0x85EBCA77u; h ^= h >> 13;
        const uint64_t nr = (l ^ h) & mask;
        l = r; r = nr;
    }
    return (l << f.half_bits) | r;
}
// minibatch row -> flat sample index: explicit table or Feistel permutation (n = invalid)
__host__ __device__ inline uint64_t feistel_permute(uint64_t i, const FeistelKey& f);
__device__ inline uint64_t minibatch_row(const int64_t* row_index, uint64_t i, const FeistelKey& f) {
    if (row_index) {
        const int64_t v = row_index[i];
        return (v >= 0 && (uint64_t)v < f.n) ? (uint64_t)v : f.n;
    }
    return feistel_permute(i, f);
}
// cycle walking; bounded (P(>1024 walks) < 1e-128); returns n on give-up (caller treats as invalid)
__host__ __device__ inline uint64_t feistel_permute(uint64_t i, const FeistelKey& f) {
    uint64_t x = feistel_once(i, f);
    for (int it = 0; it < 1024 && x >= f.n; ++it) x = feistel_once(x, f);
    return x < f.n ? x : f.n;
}

// ------------------------------------------------------------------------------------------------
// wave reductions
// ------------------------------------------------------------------------------------------------
// DPP inside each 16-lane row (quad xor 1, xor 2, half-row mirror, row mirror: every lane of a row
// holds the row sum), then the four row sums through readlane; every lane returns the same total.
// The LDS-crossbar butterfly (__shfl_xor = ds_bpermute) cost ~6 dependent LDS round trips.
template <int CTRL>
__device__ inline float dpp_movf(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ inline float wave_sum(float v) {
    v += dpp_movf<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_movf<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_movf<0x141>(v);   // row_half_mirror
    v += dpp_movf<0x140>(v);   // row_mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return (r0 + r1) + (r2 + r3);
}
__device__ inline double wave_sumd(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
