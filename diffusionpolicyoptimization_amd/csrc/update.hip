// update.hip — weight gradients, time-MLP backward, minibatch statistics, optimiser, and the
// dppo_ppo_minibatch orchestration (agent/finetune/train_ppo_diffusion_agent.py:287-356).
#include <stdlib.h>
#include <mutex>
#include <vector>
#include "dppo_ppo.h"

// ---------------------------------------------------------------------------------------------
// grouped split-K weight-gradient GEMM:  G[k][n] += sum_m XT[k][m] * DT[n][m]
// (dW = X^T dH in Keras [in,out] layout). A workgroup (one per CU) owns a WK x 128 output tile
// (WK = 128: 4 waves, WK = 256: 8 waves; DWGeom) and one m-chunk; each wave holds a 64x64
// sub-tile (4x4 MFMA tiles, 64 accumulator VGPRs).
// Both operands are feature-major, so a stage of BK rows is one 128-B line per feature: the stage
// is copied global -> LDS with 16-B global_load_lds (one 1 KiB wave-instruction = 8 features) into
// a ring of RING slots, RING - 1 stages in flight: each wave waits with a counted vmcnt for
// its own copies of the oldest stage only, then one barrier (the kernel reads ~470 MB of images
// per minibatch; one stage in flight behind a vmcnt(0) barrier left it latency bound at ~2.5 TB/s).
// The LDS image is linear per wave-instruction; the bank swizzle (16-B slot = chunk ^ (feature & 7))
// is applied on the global source address, which makes the fragment reads (ds_read_b128) conflict-free.
// The k-tile-0 workgroups also produce the "extra" rows:
//   ONES   -> bias gradient  sum_m DT[n][m]
//   ONEHOT -> per-bucket sums sum_{m: seg[m]=q} DT[n][m]  (actor in-layer: in_b and d t_emb); the
//             stage's 64 seg bytes travel in the same ring slot
// Partial tiles are added with fp32 atomics (one add per element per m-chunk).
// ---------------------------------------------------------------------------------------------
enum { EXTRA_NONE = 0, EXTRA_ONES = 1, EXTRA_ONEHOT = 2 };
#define DW_MAXP 8
#define DW_TN 128            // output tile edge along N (the gradient operand's features)
// bytes per feature per stage: 128 (two MFMA k-steps, 64 bf16 rows; the default) or 64 (one k-step).
// 64-B stages halve the slot, so the same LDS holds twice the ring (6 slots of 25 KiB at WK = 256:
// 5 stages, 120 KiB, in flight, against 3 of 49 KiB: 2 stages, 96 KiB), but pay a barrier per 32
// rows: measured slower (fused minibatch 0.535 vs 0.515 ms, tools/ab_lib.sh), so 128 stays.
#ifndef DPPO_DW_LINE
#define DPPO_DW_LINE 128
#endif
#define DW_LINE DPPO_DW_LINE
#define DW_CPL (DW_LINE / 16)       // 16-B chunks per feature line
#define DW_FPI (64 / DW_CPL)        // features per 1 KiB wave-instruction
#define DW_BOPB (DW_TN * DW_LINE)   // the B (gradient) operand's stage image
static_assert(DW_LINE == 64 || DW_LINE == 128, "DPPO_DW_LINE must be 64 or 128");

// Output tile = DW_TK(WK) x 128: WK = 128 (4 waves, 2x2 of 64x64; ring of 4 slots, 3 stages in
// flight) or WK = 256 (8 waves, 4x2 of 64x64; ring of 3 slots, 2 stages in flight). The kernel is
// bound by the latency of its staged loads (Little's law over the LDS ring: about 96 KiB in flight
// per CU either way), so the 256-row tile's 1.33x MFMAs per staged byte is what it buys (the actor's
// launches; the critic's uses the 128 ring, below).
// RC caps the ring (the critic's dW runs beside the actor's time-MLP backward, whose workgroup needs
// LDS on the same CU: a 3-slot WK = 128 ring, 101 KiB, leaves it room)
template <int WK, int RC = 8> struct DWGeom {
    static constexpr int W = WK / 32;                    // waves: 4 or 8
    static constexpr int AOPB = WK * DW_LINE;            // A (activation) operand's stage image
    static constexpr int SLOT = AOPB + DW_BOPB + 1024;   // A | B | the stage's seg bytes (padded)
    static constexpr int RING0 = 160 * 1024 / SLOT < 8 ? 160 * 1024 / SLOT : 8;
    static constexpr int RING = RING0 < RC ? RING0 : RC;   // ring slots (RING - 1 in flight)
    static constexpr int AI = WK / DW_FPI / W;           // A wave-instructions per wave per stage
    static constexpr int BI = DW_TN / DW_FPI / W;        // B wave-instructions per wave per stage
    static_assert(RING * SLOT <= 160 * 1024, "dW ring exceeds the CU's LDS");
};

struct DWProb {
    const void* XT; const void* DT; float* G; float* Gx;
    int Kx, N, extra, ktiles, ntiles;
};
struct DWArgs {
    DWProb p[DW_MAXP];
    int tile_start[DW_MAXP + 1];
    int nprob, nchunks, mchunk;
    float out_scale;          // 1 / the backward seed scale (fp16 images), 1 otherwise
    size_t ldm;
    const int8_t* seg;
    const int* rows_dev;      // non-null: only the first ceil64(*rows_dev) rows are summed (the chunk
                              // edge is recomputed on the device from that count)
};

typedef __attribute__((address_space(3))) void lds_void_t;

// extra A fragment: row q of [ones] or [one-hot(seg == q)] over EPL consecutive rows; the
// chunk's seg bytes sit in LDS (staged before the glds pipeline starts)
template <class P>
__device__ inline u32x4 extra_frag(int extra, int q, const int8_t* seg_lds) {
    using AT = typename P::AT;
    AT e[P::EPL];
    if (extra == EXTRA_ONES) {
#pragma unroll
        for (int i = 0; i < P::EPL; ++i) e[i] = P::cvt(1.f);
    } else {   // EPL bytes in one LDS read (8-B / 4-B aligned by construction)
        const uint64_t w = P::EPL == 8 ? *reinterpret_cast<const uint64_t*>(seg_lds)
                                       : (uint64_t)*reinterpret_cast<const uint32_t*>(seg_lds);
#pragma unroll
        for (int i = 0; i < P::EPL; ++i) e[i] = P::cvt((int)(int8_t)(w >> (8 * i)) == q ? 1.f : 0.f);
    }
    return __builtin_bit_cast(u32x4, e);
}

// 16-B slot of chunk c of feature f in a staged line: a bank swizzle that makes the fragment reads
// (ds_read_b128: 16 features x 4 chunks per wave-instruction, serviced in 4 lane groups of 16)
// conflict-free. 128-B lines: c ^ (f & 7). 64-B lines (4 slots, 4 features per 256-B bank row):
// c ^ H[(f >> 2) & 3] with H = {0, 2, 3, 1} gives the 16 lanes of every ds_read_b128 lane group
// ({0-3,12-15,20-27}, ...: MI355X_MICROARCH.md LDS table) 16 distinct banks.
__device__ inline int dw_swz(int f, int c) {
    if constexpr (DW_LINE == 128) return c ^ (f & 7);
    else return c ^ ((0x78 >> (2 * ((f >> 2) & 3))) & 3);   // H packed 2 bits each: 0b01_11_10_00
}
// fragment of a staged operand: feature f (within the tile), 16-B chunk c
__device__ inline u32x4 dw_lds_frag(const uint8_t* img, int f, int c) {
    return *reinterpret_cast<const u32x4*>(img + f * DW_LINE + (dw_swz(f, c) << 4));
}

// wait until at most N of this wave's vector-memory operations are outstanding
template <int N>
__device__ inline void vm_wait() {
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}

// the main loop, with or without the extra (bias / bucket) rows: two straight copies, so the
// register allocator sees one uniform accumulator set per loop (a data-dependent MFMA inside
// one loop made hipcc shuttle the accumulators between AGPRs and VGPRs every k-step).
// SEGLD: this wave also copies the stage's seg bytes (ONEHOT extra rows).
template <class P, int WK, int RC, bool EXTRA, bool SEGLD>
__device__ __forceinline__ void dw_loop(uint8_t* smem, const DWArgs& a, const DWProb& pr, int nst, size_t m_begin,
                                        int wave, int lane, const typename P::AT* const (&srcA)[DWGeom<WK, RC>::AI],
                                        const typename P::AT* const (&srcB)[DWGeom<WK, RC>::BI],
                                        f32x4 (&acc)[4][4], f32x4 (&acce)[4]) {
    using G = DWGeom<WK, RC>;
    constexpr int BK = DW_LINE / (int)sizeof(typename P::AT);
    constexpr int OPS = G::AI + G::BI + (SEGLD ? 1 : 0);      // vector-memory ops per stage per wave
    const int wr = wave >> 1, wc = wave & 1;
    const int fr = lane & 15, cq = lane >> 4;
    auto issue = [&](int st) {
        uint8_t* base = smem + (st % G::RING) * G::SLOT;
        const size_t off = (size_t)st * BK;
#pragma unroll
        for (int i = 0; i < G::AI; ++i)
            __builtin_amdgcn_global_load_lds((void*)(srcA[i] + off), (lds_void_t*)(base + (wave + G::W * i) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int i = 0; i < G::BI; ++i)
            __builtin_amdgcn_global_load_lds((void*)(srcB[i] + off),
                                             (lds_void_t*)(base + G::AOPB + (wave + G::W * i) * 1024), 16, 0, 0);
        if constexpr (SEGLD) {   // BK seg bytes, 4 per lane (lanes past BK/4 fetch bytes nobody reads)
            const int8_t* sg = a.seg + m_begin + off + 4 * (lane < BK / 4 ? lane : 0);
            __builtin_amdgcn_global_load_lds((void*)sg, (lds_void_t*)(base + G::AOPB + DW_BOPB), 4, 0, 0);
        }
    };
#pragma unroll
    for (int p = 0; p < G::RING - 1; ++p)
        if (p < nst) issue(p);
    for (int st = 0; st < nst; ++st) {
        // this wave's copies of stage st have landed once at most (stages issued after it) * OPS
        // operations are outstanding; the barrier then covers every wave's copies, and every wave
        // has finished reading stage st - 1, whose slot the next issue reuses
        const int ahead = nst - 1 - st;
        if (ahead >= G::RING - 2) vm_wait<(G::RING - 2) * OPS>();
        else if (ahead == 1) vm_wait<OPS>();
        else vm_wait<0>();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (st + G::RING - 1 < nst) issue(st + G::RING - 1);
        const uint8_t* imA = smem + (st % G::RING) * G::SLOT;
        const uint8_t* imB = imA + G::AOPB;
        const int8_t* seg_lds = (const int8_t*)(imB + DW_BOPB);
#pragma unroll
        for (int ks = 0; ks < DW_LINE / 64; ++ks) {
            u32x4 A[4], B[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                A[i] = dw_lds_frag(imA, wr * 64 + i * 16 + fr, ks * 4 + cq);
                B[i] = dw_lds_frag(imB, wc * 64 + i * 16 + fr, ks * 4 + cq);
            }
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = P::mma(A[i], B[j], acc[i][j]);
            if constexpr (EXTRA) {
                const u32x4 AE = extra_frag<P>(pr.extra, fr, seg_lds + ks * P::KG + cq * P::EPL);
#pragma unroll
                for (int j = 0; j < 4; ++j) acce[j] = P::mma(AE, B[j], acce[j]);
            }
        }
    }
}

static int dw_device_cus() {
    static int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            c = 256;
        return c > 0 ? c : 256;
    }();
    return n;
}

template <class P, int WK, int RC>
__global__ __launch_bounds__(WK / 32 * 64) void dw_kernel(DWArgs a) {   // DWGeom::W waves
    using AT = typename P::AT;
    using G = DWGeom<WK, RC>;
    constexpr int BK = DW_LINE / (int)sizeof(AT);     // rows per stage: 32 bf16 / 16 fp32 (64-B lines)
    constexpr int EPC = 16 / (int)sizeof(AT);         // elements per 16-B chunk
    // one LDS object (a second __shared__ array can make hipcc drain the glds queue at every
    // fragment read): the ring of [A | B | seg] stage slots
    __shared__ __attribute__((aligned(1024))) uint8_t smem[G::RING * G::SLOT];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // XCD-aware order: block b runs on XCD b % 8; XCD x takes the contiguous logical range
    // [x*per, (x+1)*per) of the chunk-major order, so the tiles that share one m-chunk's operand
    // slabs run together on one XCD and re-read them from its L2 instead of HBM/MALL.
    const int tiles_all = a.tile_start[a.nprob];
    const int total = tiles_all * a.nchunks;
    const int per = (total + 7) >> 3;
    const int lg = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    if (lg >= total) return;
    const int chunk = lg / tiles_all;
    const int tile = lg % tiles_all;
    int pi = 0;
    while (pi + 1 < a.nprob && tile >= a.tile_start[pi + 1]) ++pi;
    const DWProb& pr = a.p[pi];
    const int lt = tile - a.tile_start[pi];
    const int kt = lt / pr.ntiles, nt = lt % pr.ntiles;
    const int k_base = kt * WK, n_base = nt * DW_TN;
    const int wr = wave >> 1, wc = wave & 1;
    size_t lim = a.ldm, mchunk = (size_t)a.mchunk;
    if (a.rows_dev) {
        const size_t d64 = (size_t)(__builtin_amdgcn_readfirstlane(*a.rows_dev) + 63) / 64 * 64;
        lim = d64 < lim ? d64 : lim;
        mchunk = (lim + (size_t)a.nchunks * 64 - 1) / ((size_t)a.nchunks * 64) * 64;
    }
    const size_t m_begin = (size_t)chunk * mchunk;
    const size_t m_end = m_begin + mchunk < lim ? m_begin + mchunk : lim;
    if (m_begin >= m_end) return;
    const int nst = (int)((m_end - m_begin) / BK);
    const AT* XT = (const AT*)pr.XT;
    const AT* DT = (const AT*)pr.DT;
    const bool wg_extra = pr.extra != EXTRA_NONE && kt == 0;      // uniform over the workgroup
    const bool do_extra = wg_extra && wr == 0;
    const bool seg_ld = do_extra && pr.extra == EXTRA_ONEHOT;

    // per-lane glds sources of this wave's A and B wave-instructions (features ins*8 + lane/8)
    const AT* srcA[G::AI];
    const AT* srcB[G::BI];
#pragma unroll
    for (int i = 0; i < G::AI; ++i) {
        const int f = (wave + G::W * i) * DW_FPI + lane / DW_CPL;
        const int c = dw_swz(f, lane % DW_CPL);
        int fa = k_base + f; fa = fa < pr.Kx ? fa : pr.Kx - 1;
        srcA[i] = XT + (size_t)fa * a.ldm + m_begin + c * EPC;
    }
#pragma unroll
    for (int i = 0; i < G::BI; ++i) {
        const int f = (wave + G::W * i) * DW_FPI + lane / DW_CPL;
        const int c = dw_swz(f, lane % DW_CPL);
        int fb = n_base + f; fb = fb < pr.N ? fb : pr.N - 1;
        srcB[i] = DT + (size_t)fb * a.ldm + m_begin + c * EPC;
    }
    f32x4 acc[4][4], acce[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        zero_acc(acce[i]);
#pragma unroll
        for (int j = 0; j < 4; ++j) zero_acc(acc[i][j]);
    }
    // the other waves of an extra tile run the plain loop; the barrier count per stage is identical
    if (seg_ld) dw_loop<P, WK, RC, true, true>(smem, a, pr, nst, m_begin, wave, lane, srcA, srcB, acc, acce);
    else if (do_extra) dw_loop<P, WK, RC, true, false>(smem, a, pr, nst, m_begin, wave, lane, srcA, srcB, acc, acce);
    else dw_loop<P, WK, RC, false, false>(smem, a, pr, nst, m_begin, wave, lane, srcA, srcB, acc, acce);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n_base + wc * 64 + j * 16 + ccol(lane);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int k = k_base + wr * 64 + i * 16 + crow(lane, r);
                if (k < pr.Kx && n < pr.N) atomicAdd(pr.G + (size_t)k * pr.N + n, acc[i][j][r] * a.out_scale);
            }
        }
    if (do_extra) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n_base + wc * 64 + j * 16 + ccol(lane);
            if (n >= pr.N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int q = crow(lane, r);
                if (pr.extra == EXTRA_ONES) {
                    if (q == 0) atomicAdd(pr.Gx + n, acce[j][r] * a.out_scale);
                } else {
                    atomicAdd(pr.Gx + (size_t)q * pr.N + n, acce[j][r] * a.out_scale);
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// time-MLP backward (mlp_diffusion.py:40-45) from the per-t bucket sums of dh1:
//   in_b' = sum_q G[q];  dtemb[q] = G[q] . W_in[XD:XD+TD]^T;  then Dense/mish/Dense backward.
// ---------------------------------------------------------------------------------------------
#ifndef TB_THREADS
#define TB_THREADS 1024
#endif
// l2's weight gradient through the linear out layer (mlp.py:186-206: h3 = l2(.) + h1 feeds
// output_layer and nothing else, so dh3 = dy W_out^T with the out-Dense's rounded W_out, as B4 of
// the row tile forms it): dW_l2[h][j] = sum_q pl2[h][q] rnd(W_out[j][q]) with pl2 = u2^T dy from the
// dW GEMM, db_l2[j] = sum_q db_out[q] rnd(W_out[j][q]). Replaces an [H x rows] dh3 image (written by
// the row tile, read back by the dW GEMM) and an H x H x rows GEMM by an H x N x rows one.
struct L2Back {
    const float* pl2;     // [H][N]
    const float* gob;     // [N] db_out (final: the dW launch before this one produced it)
    const uint8_t* wimg;  // the packed W_OUT image ([K = H][N] in fragment order, operands rounded)
    float* gw;            // [H][H] dW_l2
    float* gb;            // [H] db_l2
    int H, N, prec;       // prec: DPPO_BF16 / DPPO_F16 (2-byte fragments) or fp32
    // critic: the minibatch's sample counts to zero afterwards (cnt[crow_n[r]], r < *crow_cnt), or null
    uint32_t* zcnt;
    const int* zlist;
    const int* zn;
};
// element (k, n) of a packed [K][N] weight image (dppo_layout.h; pack_all_kernel's slot order)
__device__ inline float packed_elem(const uint8_t* img, int K, int k, int n, int prec) {
    const bool two = prec == DPPO_BF16 || prec == DPPO_F16;
    const int KG = two ? 32 : 16, EPL = two ? 8 : 4;
    const int lane = (n & 15) + 16 * ((k % KG) / EPL);
    const size_t slot = ((size_t)(n >> 4) * packed_ksteps(K, KG) + k / KG) * 64 + lane;
    const uint8_t* e = img + slot * 16 + (size_t)(k % EPL) * (two ? 2 : 4);
    if (prec == DPPO_BF16) return (float)*(const __bf16*)e;
    if (prec == DPPO_F16) return (float)*(const _Float16*)e;
    return *(const float*)e;
}
// the same with the precision a compile-time constant: no branch between the loads (a per-element
// precision switch made hipcc wait vmcnt(0) after every 2-byte load)
template <int PREC>
__device__ inline float packed_elem_t(const uint8_t* img, int K, int k, int n) {
    constexpr bool two = PREC == DPPO_BF16 || PREC == DPPO_F16;
    constexpr int KG = two ? 32 : 16, EPL = two ? 8 : 4;
    const int lane = (n & 15) + 16 * ((k % KG) / EPL);
    const size_t slot = ((size_t)(n >> 4) * packed_ksteps(K, KG) + k / KG) * 64 + lane;
    const uint8_t* e = img + slot * 16 + (size_t)(k % EPL) * (two ? 2 : 4);
    if constexpr (PREC == DPPO_BF16) return (float)*(const __bf16*)e;
    else if constexpr (PREC == DPPO_F16) return (float)*(const _Float16*)e;
    else return *(const float*)e;
}
// Workgroup b forms rows [L2B_ROWS b, +L2B_ROWS) of dW_l2 (workgroup 0 also db_l2): thread t owns
// columns j = t, t + 256, ... with rnd(W_out[j][:]) in registers; the workgroup's pl2 rows are
// loaded up front (uniform addresses: one round trip for all of them, not one per row). No LDS and
// a few hundred FMAs per thread, so the launch fits beside the other stream's row tiles. (r03: inside
// time_bwd's single workgroup the H x H x N products took 210 us; as extra workgroups of that launch,
// inheriting its dynamic LDS, they waited for CUs, 48 us; one row's loads at a time, 33 us. r04's
// time_l2_bwd_kernel nevertheless runs them as extra workgroups of time_bwd's launch — one launch
// fewer on the chain measured faster at 6,250 rows, profiles/r04l_tail_ab.txt — and is used only by
// the default step path (DPPO_FUSED_STEP=critic) below 16,384 rows. Since ABI 12 the one-launch actor step
// runs the time-MLP backward itself and l2_back, when materialised, is this LDS-free launch alone.)
constexpr int L2B_ROWS = 4;   // rows h of dW_l2 per workgroup
constexpr int L2B_MAXN = 32;
template <int PREC, int NJ, int NQ>
__device__ inline void l2_back_cols(const L2Back& a, int b, int t, int nt) {
    // branch-free loads (a conditional load made hipcc wait for it alone): N is the instantiation's
    // width for the cfgs' widths (l2_back_rows_p), the workgroup's rows exist (b < H / L2B_ROWS), column
    // indices past H are clamped and their stores masked
    const int H = a.H, N = NQ < L2B_MAXN ? NQ : a.N;
    const int h0 = L2B_ROWS * b;
    float pv[L2B_ROWS + 1][NQ];   // the workgroup's pl2 rows, then db_out (stored by workgroup 0)
#pragma unroll
    for (int r = 0; r < L2B_ROWS; ++r)
#pragma unroll
        for (int q = 0; q < NQ; ++q) pv[r][q] = q < N ? a.pl2[(size_t)(h0 + r) * N + q] : 0.f;
#pragma unroll
    for (int q = 0; q < NQ; ++q) pv[L2B_ROWS][q] = q < N ? a.gob[q] : 0.f;
    // both columns' W_out values up front when they fit the registers (NQ <= 16), else one column at a
    // time (the 1024-thread time_l2_bwd workgroups have 128 VGPRs)
    constexpr int NW = NQ <= 16 ? NJ : 1;
    float w[NW][NQ];
    auto load_w = [&](int c, float* dst) {
        const int j = min(t + c * nt, H - 1);
#pragma unroll
        for (int q = 0; q < NQ; ++q) dst[q] = q < N ? packed_elem_t<PREC>(a.wimg, H, j, q) : 0.f;
    };
    if constexpr (NW == NJ) {
#pragma unroll
        for (int c = 0; c < NJ; ++c) load_w(c, w[c]);
    }
#pragma unroll
    for (int c = 0; c < NJ; ++c) {
        const int j = t + c * nt;
        if constexpr (NW != NJ) load_w(c, w[0]);
        const float* wc = w[NW == NJ ? c : 0];
        if (j >= H) continue;
#pragma unroll
        for (int r = 0; r <= L2B_ROWS; ++r) {
            float sum = 0.f;
#pragma unroll
            for (int q = 0; q < NQ; ++q) sum = fmaf(pv[r][q], wc[q], sum);
            if (r < L2B_ROWS) a.gw[(size_t)(h0 + r) * H + j] = sum;
            else if (b == 0) a.gb[j] = sum;
        }
    }
}
template <int PREC, int NQ>
__device__ inline void l2_back_n(const L2Back& a, int b, int t) {   // 256 threads per row group b
    if (a.H <= 256) l2_back_cols<PREC, 1, NQ>(a, b, t, 256);
    else l2_back_cols<PREC, 2, NQ>(a, b, t, 256);
}
// the kernels below are instantiated per precision and width NQ (the action-chunk widths of the cfgs:
// hopper 12, walker2d / halfcheetah 24, the critic's 1, any other N <= 32 zero-padded to 32): a runtime
// switch made hipcc outline the bodies as calls, and the unused widths' registers spilled in the
// 1024-thread time_l2_bwd workgroups
__host__ __device__ constexpr int l2_nq(int N) { return N == 1 ? 1 : (N == 12 ? 12 : (N == 24 ? 24 : L2B_MAXN)); }
// W_out's weight gradient through the folded forward (rowtile.hip: the row tiles never form h3,
// dppo_ppo.h pa0): dW_out[f][q] = sum_g rnd(W_l2[g][f]) pl2[g][q] + sum_i rnd(W_in[i][f]) pa0[i][q] +
// (b_l2[f] + b_in[f]) db_out[q], the oracle's h3^T dy with h3 = u2 rnd(W_l2) + b_l2 + a0 rnd(W_in) + b_in.
// A group of 256 threads forms OBR rows f (4 for N <= 16, else 2: 64 partial sums per thread either
// way): thread t takes rows g = t, t + 256 of W_l2 / pl2 (OBR features in one load) and row i = t of
// W_in / pa0, all loads issued before the FMAs (one round trip; a rolled loop waited for each row in
// turn); the 64 partial sums reduce over the lanes by recursive halving and then over the 4 waves
// through LDS in a fixed order. Sized for 128 VGPRs (time_l2_bwd's 1024-thread workgroups: the first
// form, 4 rows x 32 widths, spilled 1 KB per lane there).
struct OutBack {
    const float* prm;     // the actor's flat fp32 parameters
    FlatOffsets F;
    const float* pl2;     // [H][N] (the factored l2 region of the gradients when l2 is deferred)
    const float* pa0;     // [IN][N]
    const float* gob;     // [N] db_out (final: the dW launch before this one produced it)
    float* gw;            // [H][N] dW_out
    int H, IN, N, prec;
};
static OutBack make_out_back(const Dims& D, int precision, const float* actor_params, const float* pl2, const float* pa0,
                             float* ga) {
    const FlatOffsets FA = make_flat_offsets(D.IN, D.H, D.XD, D.TD);
    return OutBack{actor_params, FA, pl2, pa0, ga + FA.out_b, ga + FA.out_w, D.H, D.IN, D.XD, precision};
}
// (of the INSTANTIATED width l2_nq(N): the host's group count must use the same width as the kernel)
__host__ __device__ constexpr int ob_rows(int N) { return N <= 16 ? 4 : 2; }
template <int PREC>
__device__ inline float round_prec(float x) {
    if constexpr (PREC == DPPO_BF16) return (float)(__bf16)x;
    else if constexpr (PREC == DPPO_F16) return (float)(_Float16)x;
    else return x;
}
template <int PREC, int NQ>
__device__ inline void out_back_n(const OutBack& a, int b, bool valid, int t, float* red) {
    constexpr int OBR = ob_rows(NQ), NQP = NQ <= 16 ? 16 : 32, V = OBR * NQP;   // V = 64
    static_assert(V == 64, "one value per lane after the halving");
    const int H = a.H, f0 = OBR * b, lane = t & 63, w = t >> 6;
    const int NE = NQ < L2B_MAXN ? NQ : a.N;   // the instantiation's width (out_back_group)
    float x[V];
#pragma unroll
    for (int v = 0; v < V; ++v) x[v] = 0.f;
    if (valid) {
        // batches of rows g = t + 512 c, t + 512 c + 256 of W_l2 / pl2, then row t of W_in / pa0
        const int nb = (H + 511) / 512;
        for (int c = 0; c <= nb; ++c) {
            constexpr int NU = 2;
            float wv[NU][OBR], pv[NU][NQ];
#pragma unroll
            for (int u = 0; u < NU; ++u) {
                const bool l2 = c < nb;
                const int g = l2 ? t + 512 * c + 256 * u : t;
                const bool ok = l2 ? g < H : (u == 0 && g < a.IN);
                const float* W = (l2 ? a.prm + a.F.l2_w : a.prm + a.F.in_w) + (size_t)(ok ? g : 0) * H + f0;
                const float* P = (l2 ? a.pl2 : a.pa0) + (size_t)(ok ? g : 0) * NE;
                if constexpr (OBR == 4) {
                    const f32x4 w4 = *(const f32x4*)W;
#pragma unroll
                    for (int r = 0; r < OBR; ++r) wv[u][r] = ok ? round_prec<PREC>(w4[r]) : 0.f;
                } else {
                    const f32x2_t w2 = *(const f32x2_t*)W;
#pragma unroll
                    for (int r = 0; r < OBR; ++r) wv[u][r] = ok ? round_prec<PREC>(w2[r]) : 0.f;
                }
#pragma unroll
                for (int q = 0; q < NQ; ++q) pv[u][q] = (ok && q < NE) ? P[q] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < NU; ++u)
#pragma unroll
                for (int r = 0; r < OBR; ++r)
#pragma unroll
                    for (int q = 0; q < NQ; ++q) x[r * NQP + q] = fmaf(wv[u][r], pv[u][q], x[r * NQP + q]);
        }
    }
    // recursive halving over the 64 lanes: each xor step a lane keeps half of its vector and adds the
    // partner's copy of that half, so 6 steps leave lane l with the sum of value l (63 lane swaps,
    // against 11 dependent DPP / readlane ops per value for a whole-wave sum each)
#pragma unroll
    for (int st = 0; st < 6; ++st) {
        const int m = 32 >> st, half = V >> (st + 1);
        const bool up = (lane & m) != 0;
#pragma unroll
        for (int i = 0; i < half; ++i) {
            const float send = up ? x[i] : x[i + half];
            const float keep = up ? x[i + half] : x[i];
            x[i] = keep + __shfl_xor(send, m, 64);
        }
    }
    red[w * V + lane] = x[0];   // lane l: value l (the kept halves' offsets sum to l)
    __syncthreads();
    if (valid && t < OBR * NE) {
        const int r = t / NE, q = t % NE, f = f0 + r, v = r * NQP + q;
        if (f < H) {
            const float s = (red[v] + red[V + v]) + (red[2 * V + v] + red[3 * V + v]);
            const float bb = a.prm[a.F.l2_b + f] + a.prm[a.F.in_b + f];
            a.gw[(size_t)f * NE + q] = fmaf(bb, a.gob[q], s);
        }
    }
}
// out_back_n: every thread of the workgroup calls it (it holds a barrier); valid = the group has rows to
// form; red: OB_RED floats of LDS for this 256-thread group

constexpr int OB_RED = 4 * 64;   // floats of LDS per 256-thread group (4 waves x 64 values)

// block b: l2_back's row group b (b < l2_blocks), then the actor's out_back group b (b < ob_groups)
template <int PREC, int NQ>
__global__ __launch_bounds__(256) void l2_back_kernel(L2Back a, int l2_blocks, OutBack ob, int ob_groups) {
    if ((int)blockIdx.x < l2_blocks) l2_back_n<PREC, NQ>(a, (int)blockIdx.x, (int)threadIdx.x);
    if constexpr (NQ > 1) {   // (the critic's N = 1 has no out_back)
        if (ob_groups > 0) {
            __shared__ float red[OB_RED];
            out_back_n<PREC, NQ>(ob, (int)blockIdx.x, (int)blockIdx.x < ob_groups, (int)threadIdx.x, red);
        }
    }
    if (a.zcnt) {   // the critic's row tiles and dW (earlier on this stream) were the counts' last readers
        const int nz = *a.zn;
        for (int r = (int)(blockIdx.x * blockDim.x + threadIdx.x); r < nz; r += (int)(gridDim.x * blockDim.x))
            a.zcnt[a.zlist[r]] = 0u;
    }
}

// One workgroup; every parameter it reads (the TD temb rows of W_in and the time MLP) is staged into
// LDS in one batch of coalesced loads at the start, so the dependent phases below run from LDS and
// the kernel pays global-load latency about twice (staging, then G) instead of once per phase.
// after_stage() runs once every staged parameter is in LDS (the one-launch actor step steps W_in's
// time-embedding rows there: their old values are read, their gradient is the dW's)
// dtemb[q][0..16) = G[q] . W_in[XD + j] for TD = 16, H = 64 NU: one wave per bucket q, its G row
// loaded in one batch, 16 partial dot products per lane, reduced over the lanes by recursive halving
// (lane bits 5..2 pick the value's j, bits 1..0 are summed last)
template <int NU>
__device__ inline void dtemb_rows(const float* g0, const float* win, float* dtemb, int KF, int wave, int lane) {
    constexpr int H = 64 * NU;
    for (int q = wave; q < KF; q += TB_THREADS / 64) {
        const float* g = g0 + q * H + lane;
        float gv[NU];
#pragma unroll
        for (int u = 0; u < NU; ++u) gv[u] = g[64 * u];
        float v[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            float s = 0.f;
#pragma unroll
            for (int u = 0; u < NU; ++u) s += gv[u] * win[j * H + 64 * u + lane];
            v[j] = s;
        }
#pragma unroll
        for (int lvl = 0; lvl < 4; ++lvl) {
            const int half = 8 >> lvl, o = 32 >> lvl;
            const bool up = (lane & o) != 0;
#pragma unroll
            for (int k = 0; k < half; ++k) {
                const float keep = up ? v[k + half] : v[k], send = up ? v[k] : v[k + half];
                v[k] = keep + __shfl_xor(send, o);
            }
        }
        float t = v[0];
        t += __shfl_xor(t, 2);
        t += __shfl_xor(t, 1);
        const int j = ((lane >> 5) & 1) * 8 + ((lane >> 4) & 1) * 4 + ((lane >> 3) & 1) * 2 + ((lane >> 2) & 1);
        if ((lane & 3) == 0) dtemb[q * 16 + j] = t;
    }
}

// timing build (-DDPPO_TB_TIMING): shader-clock cycles of each phase of the time-MLP backward as
// thread 0 sees them (barrier waits included), summed over launches (tools/bench_update.py reads them)
#ifdef DPPO_TB_TIMING
__device__ unsigned long long dppo_tb_cycles[8];
#define TBPH_START unsigned long long tb_t_ = __builtin_readcyclecounter()
#define TBPH(k)                                                                   \
    do {                                                                          \
        if (threadIdx.x == 0) {                                                   \
            const unsigned long long now_ = __builtin_readcyclecounter();         \
            atomicAdd(&dppo_tb_cycles[(k)], now_ - tb_t_);                         \
            tb_t_ = now_;                                                         \
        }                                                                         \
    } while (0)
extern "C" DPPO_API int dppo_debug_tb_cycles(unsigned long long* out, int reset) {
    DPPO_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(dppo_tb_cycles), sizeof(unsigned long long) * 8));
    if (reset) {
        unsigned long long z[8] = {};
        DPPO_HIP(hipMemcpyToSymbol(HIP_SYMBOL(dppo_tb_cycles), z, sizeof(z)));
    }
    return DPPO_OK;
}
#else
#define TBPH_START
#define TBPH(k) do {} while (0)
#endif

template <class AfterStage>
__device__ inline void time_bwd_body(const float* __restrict__ gseg, const float* prm, float* grad, const FlatOffsets& F,
                                     int XD, int TD, int H, int KF, int TS, int stage_g, float* sm, AfterStage&& after_stage) {
    float* win = sm;                    // [TD][H]   W_in rows XD .. XD+TD-1
    float* w1 = win + TD * H;           // [TD][2TD]
    float* b1 = w1 + TD * 2 * TD;       // [2TD]
    float* w2 = b1 + 2 * TD;            // [TD][2TD]: time_w2 transposed (da1's reads run along h, conflict-free)
    float* dtemb = w2 + 2 * TD * TD;    // [KF][TD]
    float* e = dtemb + KF * TD;         // [KF][TD]
    float* a1 = e + KF * TD;            // [KF][2TD]
    float* da1 = a1 + KF * 2 * TD;      // [KF][2TD]
    float* ma1 = da1 + KF * 2 * TD;     // [KF][2TD] mish(a1), once per element (time_w2's gradient reads it TD times)
    float* gs = stage_g ? ma1 + KF * 2 * TD : nullptr;   // [KF][H] copy of G when it fits
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    TBPH_START;
    // Staging: every global load of a chunk is issued before its first LDS store, so the phase pays
    // one load latency per chunk (one chunk at hopper's sizes) instead of one per array (separate
    // load-then-store loops waited out four round trips in a row)
    // in_b' = sum_q G[q] (G unstaged): thread n's KF bucket values ride in the staging batch, so the
    // sum pays no round trip of its own (clamped addresses: no branch between the loads)
    constexpr int GQ = 16;
    const bool pre_in = !gs && KF <= GQ && H <= TB_THREADS;
    float gin[GQ];
    {
        constexpr int U = 8;
        const int ng = gs ? KF * H : 0, nw = TD * H, nt = TD * 2 * TD;
        if (pre_in) {
            const int nn = tid < H ? tid : 0;
#pragma unroll
            for (int q = 0; q < GQ; ++q) gin[q] = gseg[(q < KF ? q : 0) * H + nn];
        }
        const float* wsrc = prm + F.in_w + (size_t)XD * H;
        for (int base = 0; base < ng || base < nw || base < nt; base += U * TB_THREADS) {
            float rg[U], rw[U], r1[U], r2[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = base + u * TB_THREADS + tid;
                rg[u] = i < ng ? gseg[i] : 0.f;
                rw[u] = i < nw ? wsrc[i] : 0.f;
                r1[u] = i < nt ? prm[F.time_w1 + i] : 0.f;
                r2[u] = i < nt ? prm[F.time_w2 + i] : 0.f;
            }
            const float rb = base == 0 && tid < 2 * TD ? prm[F.time_b1 + tid] : 0.f;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int i = base + u * TB_THREADS + tid;
                if (i < ng) gs[i] = rg[u];
                if (i < nw) win[i] = rw[u];
                if (i < nt) { w1[i] = r1[u]; w2[(i % TD) * 2 * TD + i / TD] = r2[u]; }
            }
            if (base == 0 && tid < 2 * TD) b1[tid] = rb;
        }
    }
    TBPH(0);
    const int half = TD / 2;
    const float lnf = logf(10000.f) / (float)(half - 1);
    for (int i = tid; i < KF * TD; i += TB_THREADS) {
        const int q = i / TD, j = i % TD;
        const float f = expf(-(float)(j % half) * lnf) * (float)(q * TS);   // bucket q = row q: t = q * TS
        e[i] = j < half ? sinf(f) : cosf(f);
    }
    if (pre_in) {
        if (tid < H) {
            float s = 0.f;
#pragma unroll
            for (int q = 0; q < GQ; ++q)
                if (q < KF) s += gin[q];
            grad[F.in_b + tid] = s;
        }
    } else if (!gs) {
        for (int n = tid; n < H; n += TB_THREADS) {   // in_b' = sum_q G[q]
            float s = 0.f;
#pragma unroll 8
            for (int q = 0; q < KF; ++q) s += gseg[q * H + n];
            grad[F.in_b + n] = s;
        }
    }
    __syncthreads();
    after_stage();
    TBPH(1);
    if (gs) {   // from the staged copy: no second global round trip
        for (int n = tid; n < H; n += TB_THREADS) {
            float s = 0.f;
#pragma unroll 8
            for (int q = 0; q < KF; ++q) s += gs[q * H + n];
            grad[F.in_b + n] = s;
        }
    }
    // dtemb[q][j] = G[q] . W_in[XD + j], G from LDS when it was staged (gs != nullptr), W_in rows from
    // LDS: for TD = 16 one wave per bucket (dtemb_rows); otherwise (and with -DDPPO_TB_DTEMB_PAIRS, the
    // A/B form) one wave per (q, j) — a G load and a whole-wave sum per pair, KF * TD / 16 rounds of
    // both per wave
#ifndef DPPO_TB_DTEMB_PAIRS
    if (TD == 16 && H == 512) {
        dtemb_rows<8>(gs ? gs : gseg, win, dtemb, KF, wave, lane);
    } else
#endif
    for (int i = wave; i < KF * TD; i += TB_THREADS / 64) {
        const int q = i / TD, j = i % TD;
        const float* g = (gs ? gs : gseg) + q * H;
        float s = 0.f;
#pragma unroll 8
        for (int n = lane; n < H; n += 64) s += g[n] * win[j * H + n];
        s = wave_sum(s);
        if (lane == 0) dtemb[i] = s;
    }
    TBPH(2);
    for (int i = tid; i < KF * 2 * TD; i += TB_THREADS) {
        const int q = i / (2 * TD), h = i % (2 * TD);
        float s = b1[h];
        for (int k = 0; k < TD; ++k) s += e[q * TD + k] * w1[k * 2 * TD + h];
        a1[i] = s;
        ma1[i] = mishf(s);
    }
    __syncthreads();
    TBPH(3);
    for (int i = tid; i < KF * 2 * TD; i += TB_THREADS) {
        const int q = i / (2 * TD), h = i % (2 * TD);
        float dm = 0.f;
        for (int j = 0; j < TD; ++j) dm += dtemb[q * TD + j] * w2[j * 2 * TD + h];
        da1[i] = dm * mish_gradf(a1[i]);
    }
    for (int i = tid; i < 2 * TD * TD; i += TB_THREADS) {            // time_w2 [2TD][TD]
        const int h = i / TD, j = i % TD;
        float s = 0.f;
        for (int q = 0; q < KF; ++q) s += ma1[q * 2 * TD + h] * dtemb[q * TD + j];
        grad[F.time_w2 + i] = s;
    }
    for (int j = tid; j < TD; j += TB_THREADS) {
        float s = 0.f;
        for (int q = 0; q < KF; ++q) s += dtemb[q * TD + j];
        grad[F.time_b2 + j] = s;
    }
    __syncthreads();
    TBPH(4);
    for (int i = tid; i < TD * 2 * TD; i += TB_THREADS) {            // time_w1 [TD][2TD]
        const int k = i / (2 * TD), h = i % (2 * TD);
        float s = 0.f;
        for (int q = 0; q < KF; ++q) s += e[q * TD + k] * da1[q * 2 * TD + h];
        grad[F.time_w1 + i] = s;
    }
    for (int h = tid; h < 2 * TD; h += TB_THREADS) {
        float s = 0.f;
        for (int q = 0; q < KF; ++q) s += da1[q * 2 * TD + h];
        grad[F.time_b1 + h] = s;
    }
    TBPH(5);
}

// time_bwd, the actor's l2_back and its out_back in one launch (all follow the actor's dW and are
// independent of each other): workgroup 0 runs the time-MLP backward, the others TB_THREADS / 256 groups
// each, group g l2_back's row group g and then out_back's group g (as many workgroups as the larger
// count needs: extra workgroups waited for CUs beside the other stream's kernels)
template <int PREC, int NQ>
__global__ __launch_bounds__(TB_THREADS) void time_l2_bwd_kernel(const float* __restrict__ gseg,
                                                          const float* __restrict__ prm, float* __restrict__ grad,
                                                          FlatOffsets F, int XD, int TD, int H, int KF, int TS,
                                                          int stage_g, L2Back l2b, int l2_groups, OutBack ob,
                                                          int ob_groups) {
    extern __shared__ __attribute__((aligned(16))) float sm[];
    if (blockIdx.x == 0) {
        time_bwd_body(gseg, prm, grad, F, XD, TD, H, KF, TS, stage_g, sm, [] {});
        return;
    }
    constexpr int per = TB_THREADS / 256;
    const int grp = ((int)blockIdx.x - 1) * per + (int)threadIdx.x / 256;
    if (grp < l2_groups) l2_back_n<PREC, NQ>(l2b, grp, (int)threadIdx.x % 256);
    if (ob_groups > 0) out_back_n<PREC, NQ>(ob, grp, grp < ob_groups, (int)threadIdx.x % 256, sm + ((int)threadIdx.x / 256) * OB_RED);
}

// the (precision, width) instantiations of the l2_back / time_l2_bwd kernels
template <int PREC>
static void launch_l2_back_p(int nq, unsigned blocks, hipStream_t s, const L2Back& l2b, int l2g, const OutBack& ob, int obg) {
    switch (nq) {
        case 1: hipLaunchKernelGGL((l2_back_kernel<PREC, 1>), dim3(blocks), dim3(256), 0, s, l2b, l2g, ob, obg); break;
        case 12: hipLaunchKernelGGL((l2_back_kernel<PREC, 12>), dim3(blocks), dim3(256), 0, s, l2b, l2g, ob, obg); break;
        case 24: hipLaunchKernelGGL((l2_back_kernel<PREC, 24>), dim3(blocks), dim3(256), 0, s, l2b, l2g, ob, obg); break;
        default: hipLaunchKernelGGL((l2_back_kernel<PREC, L2B_MAXN>), dim3(blocks), dim3(256), 0, s, l2b, l2g, ob, obg); break;
    }
}
static void launch_l2_back(int prec, unsigned blocks, hipStream_t s, const L2Back& l2b, int l2g, const OutBack& ob, int obg) {
    const int nq = l2_nq(l2b.N);
    if (prec == DPPO_BF16) launch_l2_back_p<DPPO_BF16>(nq, blocks, s, l2b, l2g, ob, obg);
    else if (prec == DPPO_F16) launch_l2_back_p<DPPO_F16>(nq, blocks, s, l2b, l2g, ob, obg);
    else launch_l2_back_p<DPPO_F32>(nq, blocks, s, l2b, l2g, ob, obg);
}
template <int PREC>
static const void* time_l2_bwd_fn_p(int nq) {
    return nq == 12 ? (const void*)time_l2_bwd_kernel<PREC, 12> : nq == 24 ? (const void*)time_l2_bwd_kernel<PREC, 24>
         : (const void*)time_l2_bwd_kernel<PREC, L2B_MAXN>;
}
static const void* time_l2_bwd_fn(int prec, int nq) {
    return prec == DPPO_BF16 ? time_l2_bwd_fn_p<DPPO_BF16>(nq) : prec == DPPO_F16 ? time_l2_bwd_fn_p<DPPO_F16>(nq)
                                                                                : time_l2_bwd_fn_p<DPPO_F32>(nq);
}

// dynamic LDS of time_bwd_body over nb buckets; *stage_g = whether the bucket sums are staged too
static size_t time_bwd_lds(const Dims& D, int nb, int* stage_g) {
    size_t tsm = sizeof(float) * ((size_t)D.TD * D.H + 4 * (size_t)D.TD * D.TD + 2 * D.TD +
                                  (size_t)nb * (2 * D.TD + 3 * 2 * D.TD));
    // the bucket sums are staged only when the workgroup stays small enough to share a CU with the
    // critic's dW (its 101 KiB ring): waiting for a CU cost more than the extra global round trip
    // (staging whenever it fits, the r04 form, measured slower in r05)
    const size_t cap = 56 * 1024;
    *stage_g = tsm + sizeof(float) * (size_t)nb * D.H <= cap;
    if (*stage_g) tsm += sizeof(float) * (size_t)nb * D.H;
    return tsm;
}

// ---------------------------------------------------------------------------------------------
// minibatch advantage statistics {count, sum, sumsq} (for norm_adv, diffusion_ppo.py:74-75)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void adv_stats_kernel(const float* __restrict__ adv, FeistelKey fk, int KF, int64_t start,
                                                        int rows, const int64_t* __restrict__ row_index,
                                                        double* __restrict__ stats) {
    __shared__ double sh[3][4];
    double c = 0.0, s = 0.0, s2 = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < rows; i += (int64_t)gridDim.x * 256) {
        const uint64_t idx = minibatch_row(row_index, (uint64_t)(start + i), fk);
        if (idx >= fk.n) continue;
        const double v = adv[idx / KF];
        c += 1.0; s += v; s2 += v * v;
    }
    c = wave_sumd(c); s = wave_sumd(s); s2 = wave_sumd(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = c; sh[1][w] = s; sh[2][w] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(stats + 0, sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3]);
        atomicAdd(stats + 1, sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3]);
        atomicAdd(stats + 2, sh[2][0] + sh[2][1] + sh[2][2] + sh[2][3]);
    }
}

// the advantage moments of every minibatch of an update phase in one launch: blockIdx.y = minibatch
// m = epoch * nbatch + batch; rows [batch * rows_full, min(+rows_full, total)) of epoch `epoch`'s
// permutation (the per-minibatch adv_stats_kernel, batched)
#define ADV_MAXE 64
struct AdvStatsAll {
    FeistelKey fk[ADV_MAXE];
    int nbatch, KF;
    int64_t rows_full, total;
};
__global__ __launch_bounds__(256) void adv_stats_all_kernel(const float* __restrict__ adv, AdvStatsAll a,
                                                            double* __restrict__ stats) {
    __shared__ double sh[3][4];
    const int m = blockIdx.y, e = m / a.nbatch, b = m % a.nbatch;
    const int64_t start = (int64_t)b * a.rows_full;
    const int64_t end = start + a.rows_full < a.total ? start + a.rows_full : a.total;
    const FeistelKey fk = a.fk[e];
    double c = 0.0, s = 0.0, s2 = 0.0;
    for (int64_t i = start + (int64_t)blockIdx.x * 256 + threadIdx.x; i < end; i += (int64_t)gridDim.x * 256) {
        const uint64_t idx = minibatch_row(nullptr, (uint64_t)i, fk);
        if (idx >= fk.n) continue;
        const double v = adv[idx / a.KF];
        c += 1.0; s += v; s2 += v * v;
    }
    c = wave_sumd(c); s = wave_sumd(s); s2 = wave_sumd(s2);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = c; sh[1][w] = s; sh[2][w] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicAdd(stats + 3 * m + 0, sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3]);
        atomicAdd(stats + 3 * m + 1, sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3]);
        atomicAdd(stats + 3 * m + 2, sh[2][0] + sh[2][1] + sh[2][2] + sh[2][3]);
    }
}

// zero up to 4 byte ranges (4-B aligned, sizes multiple of 4) in one launch
struct ZeroArgs { void* p[4]; size_t n[4]; };
// 16-B stores over the 16-B aligned body of each range, 4-B stores over its head and tail (the
// grid is small: it runs while the other stream's row tiles hold most CUs)
__global__ __launch_bounds__(256) void zero_kernel(ZeroArgs z) {
    const size_t stride = (size_t)gridDim.x * 256, t0 = (size_t)blockIdx.x * 256 + threadIdx.x;
    for (int r = 0; r < 4; ++r) {
        if (!z.p[r]) continue;
        uint32_t* q = (uint32_t*)z.p[r];
        const size_t n = z.n[r] / 4;
        const size_t head = ((16 - ((uintptr_t)q & 15)) & 15) / 4 < n ? ((16 - ((uintptr_t)q & 15)) & 15) / 4 : n;
        const size_t n4 = (n - head) / 4;
        uint4* q4 = (uint4*)(q + head);
        for (size_t i = t0; i < n4; i += stride) q4[i] = uint4{0u, 0u, 0u, 0u};
        for (size_t i = t0; i < head; i += stride) q[i] = 0u;
        for (size_t i = head + 4 * n4 + t0; i < n; i += stride) q[i] = 0u;
    }
}

// ---------------------------------------------------------------------------------------------
// The critic's distinct samples of a minibatch. The value loss depends on the sample only (obs,
// returns: diffusion_ppo.py:108-118), and a minibatch of b rows drawn from S*E*K' (sample, step)
// pairs holds each sample ~b/(S*E) times (1.56x at the bench shape: 50,000 rows, 26k distinct
// samples), so the critic runs once per distinct sample with the multiplicity as the row weight:
// the same loss and gradient sums, ~half the critic row tiles and dW rows.
// crit_rows_kernel (one launch): cnt[sample] += 1 per row; the row that takes a count from 0 appends
// the sample to crow_n (one atomic per wave on crow_cnt: the wave's first-touch lanes are ranked by
// mbcnt). The list is in arrival order, so the critic's fp32 sums are accumulated in a run-dependent
// order, as the dW's split-K atomics already are. The critic's row tile reads the weights from cnt;
// the critic's last kernel (l2_back_kernel) zeroes the listed counts for the next minibatch.
// (It replaced a count launch + a one-workgroup ordered compaction: 6 + 27 us alone, 85 + 90 us
// beside the actor's row tiles.)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void crit_rows_kernel(const int64_t* __restrict__ row_index, int64_t start, int rows,
                                                        FeistelKey fk, int KF, uint32_t* __restrict__ cnt,
                                                        int* __restrict__ crow_n, int* __restrict__ crow_cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t n_iter = ((int64_t)rows + (int64_t)gridDim.x * 256 - 1) / ((int64_t)gridDim.x * 256);
    for (int64_t it = 0; it < n_iter; ++it) {   // uniform trip count: every lane reaches the ballot
        const int64_t i = (it * gridDim.x + blockIdx.x) * 256 + threadIdx.x;
        int s = -1;
        if (i < rows) {
            const uint64_t idx = minibatch_row(row_index, (uint64_t)(start + i), fk);
            if (idx < fk.n) s = (int)(idx / (uint64_t)KF);
        }
        const bool first = s >= 0 && atomicAdd(cnt + s, 1u) == 0u;
        const uint64_t m = __ballot(first);
        if (m == 0) continue;
        const int leader = __builtin_ctzll(m);
        int base = 0;
        if (lane == leader) base = atomicAdd(crow_cnt, __popcll(m));
        base = __shfl(base, leader, 64);
        if (first) crow_n[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = s;
    }
}

// Per-(device, stream) device scratch that kernels leave zeroed between uses (the fused steps' ticket
// counters, crit_rows_kernel's sample counts), created zeroed on first use and kept for the process:
// one process-wide table under a mutex, keyed by the stream's OWN device (not the caller's current
// one) and a kind. No eviction, so no device-wide wait: a pipelined sampler launch may be waiting for
// an observation the host publishes later. Growth waits for that stream alone (the only one that
// used the buffer).
enum { SCRATCH_TICKET = 0, SCRATCH_CRIT_COUNT = 1 };
static int stream_scratch(hipStream_t s, int kind, size_t bytes, void** out) {
    struct Ent { int dev; hipStream_t s; int kind; void* p; size_t cap; };
    static std::mutex mu;
    static std::vector<Ent> ents;
    int dev = 0;
    DPPO_HIP(hipStreamGetDevice(s, &dev));
    std::lock_guard<std::mutex> lk(mu);
    size_t i = 0;
    while (i < ents.size() && !(ents[i].dev == dev && ents[i].s == s && ents[i].kind == kind)) ++i;
    if (i < ents.size() && ents[i].cap >= bytes) { *out = ents[i].p; return DPPO_OK; }
    int cur = 0;
    DPPO_HIP(hipGetDevice(&cur));
    if (cur != dev) DPPO_HIP(hipSetDevice(dev));
    hipError_t err = hipSuccess;
    if (i < ents.size()) {   // grow: the old buffer's last user is this stream
        err = hipStreamSynchronize(s);
        if (err == hipSuccess) (void)hipFree(ents[i].p);
        ents.erase(ents.begin() + (ptrdiff_t)i);
    }
    void* p = nullptr;
    if (err == hipSuccess) err = hipMalloc(&p, bytes);
    if (err == hipSuccess) err = hipMemsetAsync(p, 0, bytes, s);
    if (cur != dev) (void)hipSetDevice(cur);
    if (err != hipSuccess) {
        if (p) (void)hipFree(p);
        (void)hipGetLastError();
        return dppo_set_error(DPPO_EHIP, "stream scratch (kind %d, %zu B): %s", kind, bytes, hipGetErrorString(err));
    }
    ents.push_back(Ent{dev, s, kind, p, bytes});
    *out = p;
    return DPPO_OK;
}

// crit_rows_kernel's per-sample counts (zero between uses), grown on demand
static int crit_count_scratch(int64_t nsamp, hipStream_t s, uint32_t** out) {
    const int64_t cap = nsamp > 65536 ? nsamp : 65536;
    return stream_scratch(s, SCRATCH_CRIT_COUNT, (size_t)cap * 4, (void**)out);
}

// DPPO_CRITIC_DEDUP=0 runs the critic per minibatch row (measurement knob)
static bool crit_dedup() {
    static const bool on = [] { const char* e = getenv("DPPO_CRITIC_DEDUP"); return !e || atoi(e) != 0; }();
    return on;
}

__global__ void feistel_kernel(int64_t first, int64_t count, FeistelKey fk, int64_t* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) {
        const uint64_t v = feistel_permute((uint64_t)(first + i), fk);
        out[i] = v < fk.n ? (int64_t)v : -1;
    }
}

// ---------------------------------------------------------------------------------------------
// AdamW over a flat fp32 buffer
// ---------------------------------------------------------------------------------------------
// DPPO_STEP_L2_FROM_PL2: the actor's l2 gradient in its factored form (DPPO_PPO_L2_DEFERRED): the
// l2 weight region of g holds pl2 [H][XD]; AdamW forms dW_l2[h][j] = sum_q pl2[h][q] rnd(W_out[j][q])
// and db_l2[j] = sum_q db_out[q] rnd(W_out[j][q]) itself, in l2_back_cols' order of operations
struct L2Virt {
    int on;
    int64_t w_off, b_off, ob_off;   // l2_w, l2_b, out_b offsets in the optimizer range
    int H, XD, prec;
    const uint8_t* wimg;            // the actor image's W_OUT segment (not rewritten before the pack launch)
};
__device__ inline float l2_virtual_grad(const float* __restrict__ g, const L2Virt& vt, int64_t i) {
    const float* pv;
    int j;
    if (i < vt.b_off) {        // weight: row h of pl2
        const int64_t e = i - vt.w_off;
        const int h = (int)(e / vt.H);
        j = (int)(e - (int64_t)h * vt.H);
        pv = g + vt.w_off + (int64_t)h * vt.XD;
    } else {                   // bias: db_out
        j = (int)(i - vt.b_off);
        pv = g + vt.ob_off;
    }
    float sum = 0.f;
    for (int q = 0; q < vt.XD; ++q) sum = fmaf(pv[q], packed_elem(vt.wimg, vt.H, j, q, vt.prec), sum);
    return sum;
}

struct AdamHP { float lr, wd, b1, b2, eps, alpha, bc1, bc2; int mode; };
__device__ inline void adamw_elem(float& pi, float& mi, float& vi, float gi, const AdamHP& h) {
    if (h.mode == DPPO_ADAMW_KERAS) {
        // Keras 3: decoupled decay first (variable -= variable*wd*lr), then Adam with
        // m += (g-m)(1-b1); v += (g^2-v)(1-b2); p -= m*alpha/(sqrt(v)+eps), alpha = lr*sqrt(1-b2^t)/(1-b1^t)
        pi -= pi * h.wd * h.lr;
        mi += (gi - mi) * (1.f - h.b1);
        vi += (gi * gi - vi) * (1.f - h.b2);
        pi -= (mi * h.alpha) / (sqrtf(vi) + h.eps);
    } else {
        pi *= 1.f - h.lr * h.wd;
        mi = h.b1 * mi + (1.f - h.b1) * gi;
        vi = h.b2 * vi + (1.f - h.b2) * gi * gi;
        pi -= h.lr * (mi / h.bc1) / (sqrtf(vi / h.bc2) + h.eps);
    }
}
// the minibatch's metric sums ride along (dppo_optimizer_step): one launch fewer on the
// minibatch's critical path than a separate copy. With a tag, met_out[nmet] receives it after
// the sums (system-scope release), so the host polls host-mapped memory instead of recording
// and waiting on an event (a marker packet on the minibatch chain). Workgroup 0.
__device__ inline void copy_metrics(const double* met, double* met_out, int nmet, uint64_t tag) {
    if ((int)threadIdx.x < nmet) met_out[threadIdx.x] = met[threadIdx.x];
    if (tag) {
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            __hip_atomic_store(reinterpret_cast<uint64_t*>(met_out + nmet), __builtin_bit_cast(uint64_t, (double)tag),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                                    float* __restrict__ v, int64_t n, float lr, float wd, float b1, float b2,
                                                    float eps, float alpha, float bc1, float bc2, int mode,
                                                    const double* __restrict__ met, double* __restrict__ met_out, int nmet,
                                                    uint64_t tag, L2Virt vt) {
    if (blockIdx.x == 0) copy_metrics(met, met_out, nmet, tag);
    const AdamHP h = {lr, wd, b1, b2, eps, alpha, bc1, bc2, mode};
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float pi = p[i], mi = m[i], vi = v[i];
        const bool virt = vt.on && i >= vt.w_off && i < vt.b_off + vt.H;   // [l2_w | l2_b] are adjacent
        const float gi = virt ? l2_virtual_grad(g, vt, i) : g[i];
        adamw_elem(pi, mi, vi, gi, h);
        p[i] = pi; m[i] = mi; v[i] = vi;
    }
}

// ---------------------------------------------------------------------------------------------
// The fused optimizer step (ABI 11, DPPO_STEP_FUSED_PACK and/or DPPO_STEP_CLEAR_GRADS): one launch
// for AdamW + the network's image + the next minibatch's zeroing, which otherwise take three
// launches (adamw_kernel, pack_all_kernel, zero_kernel) on every minibatch's critical path:
//  * each element's thread stores its updated parameter into its slots of the images (the pack's
//    per-element values: the same RNE conversion, FuseJob in dppo_internal.h), and zeroes its
//    gradient after the read (CLEAR_GRADS);
//  * the caller's byte ranges (the next minibatch's metrics and workspace accumulators,
//    dppo_ppo_clear_ranges) are zeroed by the launch's LAST workgroup (per-XCD ticket counters), so
//    no range is cleared before every workgroup has read what it reads — the metric sums copied out
//    included, whichever ranges the caller passes.
// The actor's step with its time-MLP backward is actor_tail_kernel below (r06); it adds the W_out
// elements the virtual l2 gradient reads; a critic's step is this kernel.
// ---------------------------------------------------------------------------------------------
struct StepFuse {
    int njobs;
    FuseJob j[FUSE_MAXJ];
    int clear_grads;
    void* clr[4];
    uint32_t clr_words[4];
    unsigned* ticket;               // zero between launches (the last workgroup resets it); null: no clears
};

template <class ET, int KG, int EPL>
__device__ inline void fuse_store(const FuseJob& J, int64_t e, float x) {
    if (J.kind == 2) {
        reinterpret_cast<float*>(J.dst)[e] = x;
        return;
    }
    // e < 2^31 (one weight tensor): 32-bit division
    int k, nn;
    if (J.kind == 0) { k = (int)e / J.IN; nn = (int)e - k * J.IN; }
    else { nn = (int)e / J.IK; k = (int)e - nn * J.IK; }
    const size_t slot = ((size_t)(nn >> 4) * J.KS + k / KG) * 64 + (nn & 15) + 16 * ((k % KG) / EPL);
    reinterpret_cast<ET*>(J.dst + slot * 16)[k % EPL] = (ET)x;
}
template <class ET, int KG, int EPL>
__device__ inline void fuse_all(const FuseJob* jobs, int njobs, int64_t i, float x) {
#pragma unroll 1
    for (int q = 0; q < njobs; ++q) {
        const FuseJob& J = jobs[q];
        if (i >= J.lo && i < J.hi) fuse_store<ET, KG, EPL>(J, i - J.lo, x);
    }
}

__device__ inline bool in_range(int64_t i, const int64_t* r) { return i >= r[0] && i < r[1]; }

// true in exactly one workgroup, the last to arrive (thread 0's view broadcast through LDS); the
// counters are per XCD first (blockIdx % 8), so no single address takes more than ~1/8 of the
// atomics, and the last workgroup resets them for the next launch on the stream
__device__ inline bool last_workgroup(unsigned* ticket) {
    __shared__ int last;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned xcd = blockIdx.x & 7, per = (gridDim.x - xcd + 7) / 8;   // blocks counted on this XCD's ticket
        int l = 0;
        if (atomicAdd(ticket + 16 * xcd, 1u) == per - 1) {
            ticket[16 * xcd] = 0u;
            const unsigned nx = gridDim.x < 8 ? gridDim.x : 8;
            l = atomicAdd(ticket + 128, 1u) == nx - 1;
            if (l) ticket[128] = 0u;
        }
        last = l;
    }
    __syncthreads();
    return last != 0;
}
__device__ inline void clear_words(void* const* clr, const uint32_t* words) {
    for (int r = 0; r < 4; ++r)
        for (uint32_t i = threadIdx.x; i < words[r]; i += blockDim.x) reinterpret_cast<uint32_t*>(clr[r])[i] = 0u;
}

// The job loops stay rolled: unrolled they made the kernel ~20k instructions long.
constexpr int FUSE_BLOCKS = 1024;
template <class ET, int KG, int EPL>
__global__ __launch_bounds__(256) void adamw_fused_kernel(float* __restrict__ p, float* g, float* __restrict__ m,
                                                          float* __restrict__ v, int64_t n, AdamHP h,
                                                          const double* met, double* met_out, int nmet, uint64_t tag,
                                                          StepFuse f) {
    if (blockIdx.x == 0) copy_metrics(met, met_out, nmet, tag);
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        float pi = p[i], mi = m[i], vi = v[i];
        const float gi = g[i];
        adamw_elem(pi, mi, vi, gi, h);
        p[i] = pi; m[i] = mi; v[i] = vi;
        if (f.clear_grads) g[i] = 0.f;
        fuse_all<ET, KG, EPL>(f.j, f.njobs, i, pi);
    }
    if (f.ticket && last_workgroup(f.ticket)) clear_words(f.clr, f.clr_words);
}

// ---------------------------------------------------------------------------------------------
// The actor's optimizer step as ONE coalesced launch (r05; the step without the time-MLP backward).
// r05's one-launch actor step stored each element into its image slots one 2-byte value at a time:
// two scattered stores per weight, slower than AdamW + the coalesced pack launch. Here every wave owns
// the elements of ONE 16-byte slot per lane of a weight tensor's packed image — a block of 16 outputs
// x KG inputs — steps them with AdamW, stores the slot (one coalesced 1 KiB wave store) and, through a
// wave-private LDS tile, the 64 slots the block covers in the transposed image; the remaining waves
// step the fp32 tensors (biases, time MLP) one element per lane and copy them into their fp32
// segments. The image bytes are the pack's (same (ET) conversion, zero padding). Under the virtual l2
// gradient (DPPO_STEP_L2_FROM_PL2) the W_out blocks and the zeroing of what the l2 elements read wait
// for the last workgroup; the caller's clear ranges too.
// ---------------------------------------------------------------------------------------------
struct TileMat {
    int64_t off;            // first element in the step's range
    int K, N, KS, KST;      // rows (inputs), columns (outputs), k-steps of the image and of the transposed one
    uint8_t* img;           // packed [K][N] image
    uint8_t* timg;          // packed image of the transpose ([N][K]), or null
    int nb;                 // 16-column blocks
};
struct TileCpy { int64_t lo, n; float* dst; };
constexpr int TILE_MAXM = 4, TILE_MAXC = 8, TILE_THREADS = 256;
struct TileStep {
    int nmat;
    TileMat mat[TILE_MAXM];
    int mstart[TILE_MAXM + 1];      // wave prefix over the mats the main grid steps
    int ncpy;
    TileCpy cpy[TILE_MAXC];
    int64_t cstart[TILE_MAXC + 1];  // element prefix over the copies
    int last_mat;                   // the mat the last workgroup steps (W_out under the virtual l2), or -1
    int64_t keep[2][2];             // read by every l2 element: zeroed by the last workgroup
    int clear_grads;
    void* clr[4];
    uint32_t clr_words[4];
    unsigned* ticket;
};
template <class ET, int KG, int EPL>
__device__ inline void tile_block(float* p, float* g, float* m, float* v, const AdamHP& h, const L2Virt& vt,
                                  const TileStep& a, const TileMat& M, int b, ET* tile, int lane) {
    static_assert(EPL * (int)sizeof(ET) == 16 && 4 * EPL == KG, "one 16-B slot per lane");
    const int nb = b % M.nb, kb = b / M.nb;
    const int n = 16 * nb + (lane & 15), jq = lane >> 4;
    ET val[EPL];
#pragma unroll
    for (int e = 0; e < EPL; ++e) {
        const int k = KG * kb + EPL * jq + e;
        float x = 0.f;
        if (k < M.K && n < M.N) {
            const int64_t i = M.off + (int64_t)k * M.N + n;
            float pi = p[i], mi = m[i], vi = v[i];
            const bool virt = vt.on && i >= vt.w_off && i < vt.b_off + vt.H;
            const float gi = virt ? l2_virtual_grad(g, vt, i) : g[i];
            if (a.clear_grads && !in_range(i, a.keep[0]) && !in_range(i, a.keep[1])) g[i] = 0.f;
            adamw_elem(pi, mi, vi, gi, h);
            p[i] = pi; m[i] = mi; v[i] = vi;
            x = pi;
        }
        val[e] = (ET)x;
    }
    u32x4 w;
    __builtin_memcpy(&w, val, 16);
    *reinterpret_cast<u32x4*>(M.img + ((((size_t)nb * M.KS + kb) << 6) + lane) * 16) = w;
    if (!M.timg) return;
    // the transposed image: tile[kl][nl] (KG x 16, wave-private) -> lane (kk, grp) reads row
    // kl = 16 (grp / NGRP) + kk, columns EPL ng .. EPL ng + EPL - 1, one T slot
#pragma unroll
    for (int e = 0; e < EPL; ++e) tile[(EPL * jq + e) * 16 + (lane & 15)] = val[e];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    constexpr int NGRP = 16 / EPL;
    const int kk = lane & 15, grp = lane >> 4;
    const int kl = 16 * (grp / NGRP) + kk, ng = grp % NGRP;
    const int k = KG * kb + kl, n0 = 16 * nb + EPL * ng;
    const u32x4 tv = *reinterpret_cast<const u32x4*>(tile + kl * 16 + EPL * ng);
    if (k < 16 * ((M.K + 15) / 16)) {
        const int ntp = k >> 4, ksp = n0 / KG, lanep = kk + 16 * ((n0 % KG) / EPL);
        *reinterpret_cast<u32x4*>(M.timg + ((((size_t)ntp * M.KST + ksp) << 6) + lanep) * 16) = tv;
    }
    __builtin_amdgcn_wave_barrier();   // the tile is rewritten by this wave's next block
}
template <class ET, int KG, int EPL>
__global__ __launch_bounds__(TILE_THREADS) void actor_tile_step_kernel(float* p, float* g, float* m, float* v, AdamHP h,
                                                                      const double* met, double* met_out, int nmet,
                                                                      uint64_t tag, L2Virt vt, TileStep a) {
    __shared__ __attribute__((aligned(16))) ET tiles[TILE_THREADS / 64][KG * 16];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (blockIdx.x == 0) copy_metrics(met, met_out, nmet, tag);
    const int gw = (int)blockIdx.x * (TILE_THREADS / 64) + wave;
    if (gw < a.mstart[a.nmat]) {
        int mi = 0;
        while (gw >= a.mstart[mi + 1]) ++mi;
        tile_block<ET, KG, EPL>(p, g, m, v, h, vt, a, a.mat[mi], gw - a.mstart[mi], tiles[wave], lane);
    } else {
        const int64_t e = (int64_t)(gw - a.mstart[a.nmat]) * 64 + lane;
        if (e < a.cstart[a.ncpy]) {
            int c = 0;
            while (e >= a.cstart[c + 1]) ++c;
            const int64_t local = e - a.cstart[c], i = a.cpy[c].lo + local;
            float pi = p[i], mi = m[i], vi = v[i];
            const bool virt = vt.on && i >= vt.w_off && i < vt.b_off + vt.H;
            const float gi = virt ? l2_virtual_grad(g, vt, i) : g[i];
            if (a.clear_grads && !in_range(i, a.keep[0]) && !in_range(i, a.keep[1])) g[i] = 0.f;
            adamw_elem(pi, mi, vi, gi, h);
            p[i] = pi; m[i] = mi; v[i] = vi;
            a.cpy[c].dst[local] = pi;
        }
    }
    if (!a.ticket || !last_workgroup(a.ticket)) return;
    if (a.last_mat >= 0) {
        const TileMat& M = a.mat[a.last_mat];
        const int nblk = M.nb * M.KS;
        for (int b = wave; b < nblk; b += TILE_THREADS / 64) tile_block<ET, KG, EPL>(p, g, m, v, h, vt, a, M, b, tiles[wave], lane);
        __syncthreads();   // every W_out slot read by an l2 element was read before the ticket
    }
    if (a.clear_grads)
        for (int r = 0; r < 2; ++r)
            for (int64_t i = a.keep[r][0] + threadIdx.x; i < a.keep[r][1]; i += TILE_THREADS) g[i] = 0.f;
    clear_words(a.clr, a.clr_words);
}

// per (device, stream): the fused steps' zeroed ticket counter block (launches on one stream are
// ordered, so they share it; the critic's step on the side stream has its own)
static int step_ticket(hipStream_t s, unsigned** out) {
    // 8 per-XCD counters 64 B apart, the total at 512 B
    return stream_scratch(s, SCRATCH_TICKET, 1024, (void**)out);
}

static int launch_adamw(float* params, const float* grads, float* m, float* v, int64_t n, int64_t step, float lr,
                        float weight_decay, float beta1, float beta2, float eps, int mode, const double* met,
                        double* met_out, int nmet, uint64_t tag, hipStream_t s, const L2Virt& vt = L2Virt{}) {
    DPPO_CHECK(n >= 0 && step >= 1, "dppo_adamw: n < 0 or step < 1");
    DPPO_CHECK(mode == DPPO_ADAMW_KERAS || mode == DPPO_ADAMW_TORCH, "dppo_adamw: bad mode");
    DPPO_CHECK(nmet >= 0 && nmet <= 256 && (nmet == 0 || (met && met_out)), "dppo_optimizer_step: bad metrics copy");
    DPPO_CHECK(tag == 0 || (met_out && tag < ((uint64_t)1 << 53)), "dppo_optimizer_step: a tag needs metrics_out and < 2^53");
    if (n == 0 && nmet == 0 && tag == 0) return DPPO_OK;
    DPPO_CHECK(n == 0 || (params && grads && m && v), "dppo_adamw: null pointer");
    const double bc1 = 1.0 - pow((double)beta1, (double)step);
    const double bc2 = 1.0 - pow((double)beta2, (double)step);
    const float alpha = (float)((double)lr * sqrt(bc2) / bc1);
    const int64_t blocks64 = (n + 255) / 256;
    const unsigned blocks = (unsigned)(blocks64 < 1 ? 1 : (blocks64 < 4096 ? blocks64 : 4096));
    DppoKtScope kt(KT_ADAMW, s);
    hipLaunchKernelGGL(adamw_kernel, dim3(blocks), dim3(256), 0, s, params, grads, m, v, n, lr,
                       weight_decay, beta1, beta2, eps, alpha, (float)bc1, (float)bc2, mode, met, met_out, nmet, tag, vt);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_adamw(float* params, const float* grads, float* m, float* v, int64_t n, int64_t step, float lr,
                          float weight_decay, float beta1, float beta2, float eps, int mode, void* stream) {
    return launch_adamw(params, grads, m, v, n, step, lr, weight_decay, beta1, beta2, eps, mode, nullptr, nullptr, 0, 0,
                        (hipStream_t)stream);
}

static int optimizer_step_impl(const dppo_dims* d, int precision, float* params, float* grads, float* m, float* v,
                               int64_t n, int64_t step, float lr, float weight_decay, float beta1, float beta2,
                               float eps, int mode, const float* actor_params, void* packed_actor,
                               const float* critic_params, void* packed_critic, const double* metrics,
                               double* metrics_out, int n_metrics, uint64_t metrics_tag, void* const* clear_ptrs,
                               const size_t* clear_bytes, int n_clear, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(!packed_actor == !actor_params && !packed_critic == !critic_params,
               "dppo_optimizer_step: a packed image needs its parameters");
    DPPO_CHECK(n_clear >= 0 && n_clear <= 4 && (n_clear == 0 || (clear_ptrs && clear_bytes)),
               "dppo_optimizer_step_ex: at most 4 clear ranges");
    for (int r = 0; r < n_clear; ++r)
        DPPO_CHECK(clear_ptrs[r] && ((uintptr_t)clear_ptrs[r] & 3) == 0 && clear_bytes[r] % 4 == 0 &&
                   clear_bytes[r] / 4 < ((size_t)1 << 32), "dppo_optimizer_step_ex: clear range %d must be 4-B aligned", r);
    hipStream_t s = (hipStream_t)stream;
    // metrics_out may be mapped host memory (dppo_host_alloc): the kernel stores through its
    // device address
    double* mout = metrics_out;
    if (mout) {
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, metrics_out, 0) == hipSuccess && dp) mout = (double*)dp;
        else (void)hipGetLastError();
    }
    const bool defer = (mode & DPPO_STEP_DEFER_SAMPLER_TABLES) != 0;
    const bool l2v = (mode & DPPO_STEP_L2_FROM_PL2) != 0;
    const bool fuse = (mode & DPPO_STEP_FUSED_PACK) != 0;
    const bool clear_g = (mode & DPPO_STEP_CLEAR_GRADS) != 0;
    mode &= ~(DPPO_STEP_DEFER_SAMPLER_TABLES | DPPO_STEP_L2_FROM_PL2 | DPPO_STEP_FUSED_PACK | DPPO_STEP_CLEAR_GRADS);
    const FlatOffsets FA = make_flat_offsets(D.IN, D.H, D.XD, D.TD);
    const FlatOffsets FC = make_flat_offsets(D.SD, D.HC, 1, 0);
    L2Virt vt = {};
    if (l2v) {
        DPPO_CHECK(packed_actor && actor_params == params,
                   "dppo_optimizer_step: DPPO_STEP_L2_FROM_PL2 needs the actor's image and the actor range first");
        DPPO_CHECK(n >= (int64_t)FA.count, "dppo_optimizer_step: DPPO_STEP_L2_FROM_PL2 needs the whole actor range");
        DPPO_CHECK(FA.l2_b == FA.l2_w + (size_t)D.H * D.H, "l2 layout");
        const MlpLayout L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
        vt = L2Virt{1, (int64_t)FA.l2_w, (int64_t)FA.l2_b, (int64_t)FA.out_b, D.H, D.XD, precision,
                    (const uint8_t*)packed_actor + L.off[SEG_W_OUT]};
    }
    // the one-launch form: a single network whose parameters are exactly the range. The actor's
    // (actor_tile_step_kernel) leaves its TEMB table and split-sampler tables to the fold launch (the row
    // tiles derive the time embeddings, the sampler re-derives the tables before its next launch)
    const bool one_actor = packed_actor && !packed_critic && actor_params == params && n == (int64_t)FA.count;
    const bool one_critic = packed_critic && !packed_actor && critic_params == params && n == (int64_t)FC.count;
    if (fuse && (one_actor || one_critic) && n > 0) {
        DPPO_CHECK(n_metrics >= 0 && n_metrics <= 256 && (n_metrics == 0 || (metrics && mout)),
                   "dppo_optimizer_step: bad metrics copy");
        DPPO_CHECK(metrics_tag == 0 || (mout && metrics_tag < ((uint64_t)1 << 53)),
                   "dppo_optimizer_step: a tag needs metrics_out and < 2^53");
        DPPO_CHECK(step >= 1 && (mode == DPPO_ADAMW_KERAS || mode == DPPO_ADAMW_TORCH), "dppo_adamw: bad step or mode");
        DPPO_CHECK(params && grads && m && v, "dppo_adamw: null pointer");
        const double bc1 = 1.0 - pow((double)beta1, (double)step);
        const double bc2 = 1.0 - pow((double)beta2, (double)step);
        const AdamHP h = {lr, weight_decay, beta1, beta2, eps, (float)((double)lr * sqrt(bc2) / bc1), (float)bc1,
                          (float)bc2, mode};
        if (one_critic) {
            StepFuse f = {};
            f.njobs = dppo_fuse_jobs(D.SD, D.HC, 1, 0, precision, packed_critic, 0, f.j);
            DPPO_CHECK(f.njobs >= 0, "dppo_optimizer_step: fused pack jobs");
            f.clear_grads = clear_g ? 1 : 0;
            for (int r = 0; r < n_clear; ++r) { f.clr[r] = clear_ptrs[r]; f.clr_words[r] = (uint32_t)(clear_bytes[r] / 4); }
            if (n_clear > 0) {
                rc = step_ticket(s, &f.ticket);
                if (rc) return rc;
            }
            const int64_t blocks64 = (n + 255) / 256;
            const unsigned blocks = (unsigned)(blocks64 < FUSE_BLOCKS ? blocks64 : FUSE_BLOCKS);
            DppoKtScope kt(KT_ADAMW, s);
            if (precision == DPPO_BF16)
                hipLaunchKernelGGL((adamw_fused_kernel<__bf16, 32, 8>), dim3(blocks), dim3(256), 0, s, params, grads, m, v,
                                   n, h, metrics, mout, n_metrics, metrics_tag, f);
            else if (precision == DPPO_F16)
                hipLaunchKernelGGL((adamw_fused_kernel<_Float16, 32, 8>), dim3(blocks), dim3(256), 0, s, params, grads, m,
                                   v, n, h, metrics, mout, n_metrics, metrics_tag, f);
            else
                hipLaunchKernelGGL((adamw_fused_kernel<float, 16, 4>), dim3(blocks), dim3(256), 0, s, params, grads, m, v,
                                   n, h, metrics, mout, n_metrics, metrics_tag, f);
            DPPO_HIP(hipGetLastError());
            return DPPO_OK;
        }
        FuseJob jobs[FUSE_MAXJ];
        const int nj = dppo_fuse_jobs(D.IN, D.H, D.XD, D.TD, precision, packed_actor, D.K, jobs);
        DPPO_CHECK(nj >= 0, "dppo_optimizer_step: fused pack jobs");
        TileStep t = {};
        t.last_mat = -1;
        for (int q = 0; q < nj; ++q) {
            const FuseJob& J = jobs[q];
            if (J.kind == 0) {
                DPPO_CHECK(t.nmat < TILE_MAXM, "actor tile step: too many weight tensors");
                TileMat& M = t.mat[t.nmat++];
                M.off = J.lo; M.K = J.IK; M.N = J.IN; M.KS = J.KS; M.img = J.dst; M.timg = nullptr; M.KST = 0;
                M.nb = dppo_cdiv(M.N, 16);
            } else if (J.kind == 2) {
                DPPO_CHECK(t.ncpy < TILE_MAXC, "actor tile step: too many fp32 tensors");
                t.cpy[t.ncpy++] = TileCpy{J.lo, J.hi - J.lo, (float*)J.dst};
            }
        }
        for (int q = 0; q < nj; ++q) {   // the transposed images, matched to their tensor
            const FuseJob& J = jobs[q];
            if (J.kind != 1) continue;
            int mi = 0;
            while (mi < t.nmat && t.mat[mi].off != J.lo) ++mi;
            DPPO_CHECK(mi < t.nmat && J.IK == t.mat[mi].N && J.IN == t.mat[mi].K, "actor tile step: transposed image");
            t.mat[mi].timg = J.dst; t.mat[mi].KST = J.KS;
        }
        for (int r = 0; r < 2; ++r) t.keep[r][0] = t.keep[r][1] = -1;
        if (l2v) {
            for (int mi = 0; mi < t.nmat; ++mi)
                if (t.mat[mi].off == (int64_t)FA.out_w) t.last_mat = mi;
            DPPO_CHECK(t.last_mat >= 0, "actor tile step: W_out");
            t.keep[0][0] = (int64_t)FA.l2_w; t.keep[0][1] = (int64_t)(FA.l2_w + (size_t)D.H * D.XD);
            t.keep[1][0] = (int64_t)FA.out_b; t.keep[1][1] = (int64_t)(FA.out_b + D.XD);
        }
        t.mstart[0] = 0;
        for (int mi = 0; mi < t.nmat; ++mi)
            t.mstart[mi + 1] = t.mstart[mi] + (mi == t.last_mat ? 0 : t.mat[mi].nb * t.mat[mi].KS);
        t.cstart[0] = 0;
        for (int c = 0; c < t.ncpy; ++c) t.cstart[c + 1] = t.cstart[c] + t.cpy[c].n;
        t.clear_grads = clear_g ? 1 : 0;
        for (int r = 0; r < n_clear; ++r) { t.clr[r] = clear_ptrs[r]; t.clr_words[r] = (uint32_t)(clear_bytes[r] / 4); }
        if (l2v || n_clear > 0 || clear_g) {
            rc = step_ticket(s, &t.ticket);
            if (rc) return rc;
        }
        const int64_t waves = t.mstart[t.nmat] + (t.cstart[t.ncpy] + 63) / 64;
        const unsigned blocks = (unsigned)((waves + TILE_THREADS / 64 - 1) / (TILE_THREADS / 64));
        {
            DppoKtScope kt(KT_ADAMW, s);
            if (precision == DPPO_BF16)
                hipLaunchKernelGGL((actor_tile_step_kernel<__bf16, 32, 8>), dim3(blocks), dim3(TILE_THREADS), 0, s,
                                   params, grads, m, v, h, metrics, mout, n_metrics, metrics_tag, vt, t);
            else if (precision == DPPO_F16)
                hipLaunchKernelGGL((actor_tile_step_kernel<_Float16, 32, 8>), dim3(blocks), dim3(TILE_THREADS), 0, s,
                                   params, grads, m, v, h, metrics, mout, n_metrics, metrics_tag, vt, t);
            else
                hipLaunchKernelGGL((actor_tile_step_kernel<float, 16, 4>), dim3(blocks), dim3(TILE_THREADS), 0, s,
                                   params, grads, m, v, h, metrics, mout, n_metrics, metrics_tag, vt, t);
        }
        DPPO_HIP(hipGetLastError());
        rc = dppo_pack_rt_fold(D.IN, D.H, D.XD, D.TD, precision, actor_params, packed_actor, D.K, D.TS, s);   // cross-element: not per element
        if (rc) return rc;
        return dppo_mark_tables_stale(D, precision, actor_params, packed_actor, true);
    }
    // the launch-per-stage form (any ranges and images): AdamW, then the pack, which also zeroes the
    // gradients AdamW has read (DPPO_STEP_CLEAR_GRADS) and the caller's ranges
    rc = launch_adamw(params, grads, m, v, n, step, lr, weight_decay, beta1, beta2, eps, mode, metrics, mout,
                      n_metrics, metrics_tag, s, vt);
    if (rc) return rc;
    void* zp[5];
    size_t zb[5];
    int nz = 0;
    if (clear_g && n > 0) { zp[nz] = grads; zb[nz] = (size_t)n * sizeof(float); ++nz; }
    for (int r = 0; r < n_clear; ++r) { zp[nz] = clear_ptrs[r]; zb[nz] = clear_bytes[r]; ++nz; }
    for (int r = 0; r < nz; ++r)
        DPPO_CHECK(zb[r] / 4 < ((size_t)1 << 31), "dppo_optimizer_step_ex: clear range %d too large", r);
    if (packed_actor || packed_critic)
        return dppo_pack_models(D, precision, actor_params, packed_actor, critic_params, packed_critic, s, defer, zp, zb, nz);
    if (nz) {   // no image to pack: the clears alone
        ZeroArgs z = {};
        for (int r = 0; r < nz; ++r) {
            if (r == 4) {
                hipLaunchKernelGGL(zero_kernel, dim3(16), dim3(256), 0, s, z);
                DPPO_HIP(hipGetLastError());
                z = ZeroArgs{};
            }
            z.p[r % 4] = zp[r]; z.n[r % 4] = zb[r];
        }
        DppoKtScope kt(KT_ZERO, s);
        hipLaunchKernelGGL(zero_kernel, dim3(16), dim3(256), 0, s, z);
        DPPO_HIP(hipGetLastError());
    }
    return DPPO_OK;
}

extern "C" int dppo_optimizer_step(const dppo_dims* d, int precision, float* params, const float* grads, float* m,
                                   float* v, int64_t n, int64_t step, float lr, float weight_decay, float beta1,
                                   float beta2, float eps, int mode, const float* actor_params, void* packed_actor,
                                   const float* critic_params, void* packed_critic, const double* metrics,
                                   double* metrics_out, int n_metrics, uint64_t metrics_tag, void* stream) {
    DPPO_CHECK((mode & DPPO_STEP_CLEAR_GRADS) == 0, "dppo_optimizer_step: DPPO_STEP_CLEAR_GRADS needs dppo_optimizer_step_ex");
    return optimizer_step_impl(d, precision, params, const_cast<float*>(grads), m, v, n, step, lr, weight_decay, beta1,
                               beta2, eps, mode, actor_params, packed_actor, critic_params, packed_critic, metrics,
                               metrics_out, n_metrics, metrics_tag, nullptr, nullptr, 0, stream);
}

extern "C" int dppo_optimizer_step_ex(const dppo_dims* d, int precision, float* params, float* grads, float* m,
                                      float* v, int64_t n, int64_t step, float lr, float weight_decay, float beta1,
                                      float beta2, float eps, int mode, const float* actor_params, void* packed_actor,
                                      const float* critic_params, void* packed_critic, const double* metrics,
                                      double* metrics_out, int n_metrics, uint64_t metrics_tag, void* const* clear_ptrs,
                                      const size_t* clear_bytes, int n_clear, void* stream) {
    return optimizer_step_impl(d, precision, params, grads, m, v, n, step, lr, weight_decay, beta1, beta2, eps, mode,
                               actor_params, packed_actor, critic_params, packed_critic, metrics, metrics_out,
                               n_metrics, metrics_tag, clear_ptrs, clear_bytes, n_clear, stream);
}

// ---------------------------------------------------------------------------------------------
// Learnable DDIM eta (§8(f) row 4; the original DPPO's EtaFixed, parity unpinned: the reference's
// eta module is absent and its eta step is commented out, train_ppo_diffusion_agent.py:28-45,
// 358-359). state = {logit, m, v}; eta = eta_min + (eta_max - eta_min) (tanh(logit) + 1) / 2.
// One workgroup: thread 0 applies AdamW to the logit with d loss / d logit = metrics[8] d eta / d
// logit (metrics[8] = d loss / d eta from the DPPO_PPO_LEARN_ETA row tiles), then one thread per
// DDIM row rewrites the eta-dependent schedule columns c2, c3, logvar in ddim_buffers' fp32 order of
// operations (model/diffusion/sampling.py), from the eta-independent base rows
// {abar_prev, sqrt(abar_prev), sqrt(abar), sqrt(1 - abar), s}.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void eta_step_kernel(float* __restrict__ st, const double* __restrict__ met, int apply,
                                                     float lr, float wd, float b1, float b2, float eps, float alpha,
                                                     float bc1, float bc2, int mode, float emin, float emax,
                                                     const float* __restrict__ base, float* __restrict__ sched, int S,
                                                     float* __restrict__ eta_out) {
    __shared__ float eta_s;
    if (threadIdx.x == 0) {
        float th = st[0];
        if (apply) {
            const float tn = tanhf(th);
            const float gi = (float)met[8] * (0.5f * (emax - emin) * (1.f - tn * tn));
            float mi = st[1], vi = st[2];
            if (mode == DPPO_ADAMW_KERAS) {
                th -= th * wd * lr;
                mi += (gi - mi) * (1.f - b1);
                vi += (gi * gi - vi) * (1.f - b2);
                th -= (mi * alpha) / (sqrtf(vi) + eps);
            } else {
                th *= 1.f - lr * wd;
                mi = b1 * mi + (1.f - b1) * gi;
                vi = b2 * vi + (1.f - b2) * gi * gi;
                th -= lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
            }
            st[0] = th; st[1] = mi; st[2] = vi;
        }
        const float e = emin + (emax - emin) * (0.5f * (tanhf(th) + 1.f));
        eta_s = e;
        if (eta_out) *eta_out = e;
    }
    __syncthreads();
    const int j = threadIdx.x;
    if (j < S) {
        const float* b = base + 5 * j;   // abar_prev, sqrt(abar_prev), sqrt(abar), sqrt(1 - abar), s
        const float sig = fmaxf(__fmul_rn(eta_s, b[4]), 1e-10f);
        const float in = __fsub_rn(__fsub_rn(1.f, b[0]), __fmul_rn(sig, sig));
        const float dd = sqrtf(fminf(fmaxf(in, 0.f), 1e6f));
        float* r = sched + (size_t)j * DPPO_SCHED_COLS;
        r[2] = __fsub_rn(b[1], __fdiv_rn(__fmul_rn(dd, b[2]), b[3]));
        r[3] = __fdiv_rn(dd, b[3]);
        r[4] = logf(__fmul_rn(sig, sig));
    }
}

extern "C" int dppo_eta_step(float* eta_state, const double* metrics, int64_t step, float lr, float weight_decay,
                             float beta1, float beta2, float eps, int mode, float eta_min, float eta_max,
                             const float* ddim_base, float* sched, int ddim_steps, float* eta_out, void* stream) {
    DPPO_CHECK(eta_state && ddim_base && sched, "dppo_eta_step: null pointer");
    DPPO_CHECK(ddim_steps >= 1 && ddim_steps <= 64, "dppo_eta_step: ddim_steps %d outside [1, 64]", ddim_steps);
    DPPO_CHECK(eta_max > eta_min, "dppo_eta_step: eta_max must exceed eta_min");
    DPPO_CHECK(mode == DPPO_ADAMW_KERAS || mode == DPPO_ADAMW_TORCH, "dppo_eta_step: bad mode");
    const int apply = metrics != nullptr && step >= 1;
    const double bc1 = apply ? 1.0 - pow((double)beta1, (double)step) : 1.0;
    const double bc2 = apply ? 1.0 - pow((double)beta2, (double)step) : 1.0;
    const float alpha = (float)((double)lr * sqrt(bc2) / bc1);
    hipLaunchKernelGGL(eta_step_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, eta_state, metrics, apply, lr,
                       weight_decay, beta1, beta2, eps, alpha, (float)bc1, (float)bc2, mode, eta_min, eta_max, ddim_base,
                       sched, ddim_steps, eta_out);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_pack_all(const dppo_dims* d, int precision, const float* actor_params, void* packed_actor,
                             const float* critic_params, void* packed_critic, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(!packed_actor == !actor_params && !packed_critic == !critic_params,
               "dppo_pack_all: a packed image needs its parameters");
    return dppo_pack_models(D, precision, actor_params, packed_actor, critic_params, packed_critic, (hipStream_t)stream);
}

extern "C" int dppo_feistel_permute(int64_t first, int64_t count, int64_t n, uint64_t seed, int epoch, int64_t* out,
                                    void* stream) {
    DPPO_CHECK(n > 0 && count >= 0 && first >= 0, "dppo_feistel_permute: bad range");
    if (count == 0) return DPPO_OK;
    DPPO_CHECK(out, "dppo_feistel_permute: null out");
    const FeistelKey fk = feistel_key((uint64_t)n, seed, epoch);
    hipLaunchKernelGGL(feistel_kernel, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       first, count, fk, out);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_ppo_adv_stats(const float* advantages, int64_t total, int K_ft, uint64_t perm_seed, int epoch,
                                  int64_t start, int rows, const int64_t* row_index, double* adv_stats, void* stream) {
    DPPO_CHECK(advantages && adv_stats && total > 0 && K_ft > 0 && rows >= 0, "dppo_ppo_adv_stats: bad args");
    hipStream_t s = (hipStream_t)stream;
    DPPO_HIP(hipMemsetAsync(adv_stats, 0, 3 * sizeof(double), s));
    if (rows == 0) return DPPO_OK;
    const FeistelKey fk = feistel_key((uint64_t)total, perm_seed, epoch);
    const int blocks = dppo_cdiv(rows, 256) < 512 ? dppo_cdiv(rows, 256) : 512;
    hipLaunchKernelGGL(adv_stats_kernel, dim3(blocks), dim3(256), 0, s, advantages, fk, K_ft, start, rows, row_index,
                       adv_stats);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_ppo_adv_stats_all(const float* advantages, int64_t total, int K_ft, uint64_t perm_seed, int epoch0,
                                      int n_epochs, int64_t rows_full, int n_batch, double* adv_stats, void* stream) {
    DPPO_CHECK(advantages && adv_stats && total > 0 && K_ft > 0 && rows_full > 0 && n_batch > 0 && n_epochs > 0,
               "dppo_ppo_adv_stats_all: bad args");
    DPPO_CHECK(n_epochs <= ADV_MAXE, "dppo_ppo_adv_stats_all: at most %d epochs", ADV_MAXE);
    DPPO_CHECK((uint64_t)total < ((uint64_t)1 << 32), "dppo_ppo_adv_stats_all: total exceeds 2^32");
    hipStream_t s = (hipStream_t)stream;
    const int nm = n_epochs * n_batch;
    DPPO_HIP(hipMemsetAsync(adv_stats, 0, (size_t)3 * nm * sizeof(double), s));
    AdvStatsAll a = {};
    for (int e = 0; e < n_epochs; ++e) a.fk[e] = feistel_key((uint64_t)total, perm_seed, epoch0 + e);
    a.nbatch = n_batch; a.KF = K_ft; a.rows_full = rows_full; a.total = total;
    const int64_t bx = dppo_cdiv((int)(rows_full < total ? rows_full : total), 256);
    const int blocks = bx < 64 ? (int)bx : 64;
    DppoKtScope kt(KT_ADV_STATS, s);
    hipLaunchKernelGGL(adv_stats_all_kernel, dim3(blocks, nm), dim3(256), 0, s, advantages, a, adv_stats);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" size_t dppo_ppo_workspace_bytes(const dppo_dims* d, int precision, int batch_rows) {
    Dims D;
    if (dppo_check_dims(d, &D) || batch_rows < 0) return 0;
    return make_ppo_workspace(D, precision, batch_rows, nullptr).total;
}

// wk = 256 / 128, or 0: WK = 128 with the 3-slot ring (the critic's dW beside the actor's tail)
template <class P>
static int launch_dw(const DWArgs& a, int wk, hipStream_t s) {
    const int tiles = a.tile_start[a.nprob];
    const int64_t blocks = 8 * (((int64_t)tiles * a.nchunks + 7) / 8);   // whole XCD rounds
    if (wk == 256)
        hipLaunchKernelGGL((dw_kernel<P, 256, 8>), dim3((unsigned)blocks), dim3(DWGeom<256>::W * 64), 0, s, a);
    else if (wk == 128)
        hipLaunchKernelGGL((dw_kernel<P, 128, 8>), dim3((unsigned)blocks), dim3(DWGeom<128>::W * 64), 0, s, a);
    else
        hipLaunchKernelGGL((dw_kernel<P, 128, 3>), dim3((unsigned)blocks), dim3(128 / 32 * 64), 0, s, a);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// k-tile edge of the grouped dW launches (128 measured slower, r04)
constexpr int DW_TK = 256;

// one non-blocking side stream (+ fork/join events) per device and host thread, created on first use;
// null if creation fails (the caller then runs everything on its own stream)
// (the critic's half of a whole minibatch)
struct SideStream { hipStream_t stream; hipEvent_t fork, join; };
static SideStream* side_stream() {
    constexpr int MAXDEV = 16;
    thread_local SideStream ss[MAXDEV] = {};
    thread_local bool tried[MAXDEV] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= MAXDEV) return nullptr;
    SideStream& e = ss[dev];
    if (!tried[dev]) {
        tried[dev] = true;
        if (hipStreamCreateWithFlags(&e.stream, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e.fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.join, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            e.stream = nullptr;
        }
    }
    return e.stream ? &e : nullptr;
}

// the actor's l2 weight gradient from pl2 (l2_back_kernel: no LDS, so it starts on any CU with a
// free wave slot), then the time-MLP backward over nb buckets at t = q * TS (the bucket sums in gseg)
// the actor's out_back (dW_out through the folded forward) over the pl2 / pa0 sums of the dW launch

// after the actor's dW: the time-MLP backward over nb buckets at t = q * TS (the bucket sums in gseg),
// W_out's gradient (out_back) and, unless the l2 gradient stays factored, l2's from pl2, in one launch
static int launch_time_bwd(const Dims& D, int precision, const float* gseg, const float* pl2, const float* pa0,
                           const void* packed_actor, const float* actor_params, float* ga, int nb, int TS, hipStream_t s,
                           bool l2_back = true) {
    const FlatOffsets FA = make_flat_offsets(D.IN, D.H, D.XD, D.TD);
    const MlpLayout L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    L2Back l2b = {pl2, ga + FA.out_b, (const uint8_t*)packed_actor + L.off[SEG_W_OUT], ga + FA.l2_w, ga + FA.l2_b, D.H,
                  D.XD, precision, nullptr, nullptr, nullptr};
    DPPO_CHECK(D.XD <= L2B_MAXN, "l2_back: action horizon x dim %d > %d", D.XD, L2B_MAXN);
    DPPO_CHECK(D.IN <= 256 && D.H % 4 == 0, "out_back: in_dim %d > 256", D.IN);
    // (time_bwd forked onto a side stream beside l2_back measured slower: 0.428 vs 0.406 ms per
    // minibatch, same box, tools/r03_ab2.sh; since r04 the two share one launch instead)
    int stage_g = 0;
    const size_t tsm0 = time_bwd_lds(D, nb, &stage_g);
    const size_t tsm = tsm0 > sizeof(float) * OB_RED * (TB_THREADS / 256) ? tsm0 : sizeof(float) * OB_RED * (TB_THREADS / 256);
    DPPO_CHECK(tsm <= 160 * 1024, "time_bwd: LDS staging %zu B exceeds 160 KB", tsm);
    const int per = TB_THREADS / 256;
    const int l2g = l2_back ? dppo_cdiv(D.H, L2B_ROWS) : 0, obg = dppo_cdiv(D.H, ob_rows(l2_nq(D.XD)));
    const int nq = l2_nq(D.XD);
    const void* fn = time_l2_bwd_fn(precision, nq);
    { const int rc_ = dppo_func_lds(fn, tsm); if (rc_) return rc_; }
    DppoKtScope kt(KT_TIME_BWD, s);
    const OutBack ob = make_out_back(D, precision, actor_params, pl2, pa0, ga);
    const dim3 grid(1 + dppo_cdiv(l2g > obg ? l2g : obg, per));
    int XD = D.XD, TD = D.TD, H = D.H;
    FlatOffsets fa = FA;
    const float* prm = actor_params;
    void* args[] = {(void*)&gseg, (void*)&prm, (void*)&ga, (void*)&fa, (void*)&XD, (void*)&TD, (void*)&H, (void*)&nb,
                    (void*)&TS, (void*)&stage_g, (void*)&l2b, (void*)&l2g, (void*)&ob, (void*)&obg};
    DPPO_HIP(hipLaunchKernel(fn, grid, dim3(TB_THREADS), args, tsm, s));
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// the critic's l2 weight gradient from cpl2 (N = 1)
static int launch_critic_l2_back(const Dims& D, int precision, const float* cpl2, const void* packed_critic, float* gc,
                                 uint32_t* zcnt, const int* zlist, const int* zn, hipStream_t s) {
    const FlatOffsets FC = make_flat_offsets(D.SD, D.HC, 1, 0);
    const MlpLayout L = make_mlp_layout(D.SD, D.HC, 1, 0, precision);
    L2Back l2b = {cpl2, gc + FC.out_b, (const uint8_t*)packed_critic + L.off[SEG_W_OUT], gc + FC.l2_w, gc + FC.l2_b, D.HC, 1,
                  precision, zcnt, zlist, zn};
    DppoKtScope kt(KT_L2_BACK, s);
    launch_l2_back(precision, (unsigned)dppo_cdiv(D.HC, L2B_ROWS), s, l2b, dppo_cdiv(D.HC, L2B_ROWS), OutBack{}, 0);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// the atomically accumulated outputs a minibatch half (or the whole) zeroes first: gradients (entry
// 0), metrics (actor: 0, 2..15; critic: 1), pl2 | bucket sums, cpl2 | stats | crow_cnt. Entries 1..3
// are what dppo_ppo_clear_ranges reports (the gradients are cleared by the optimizer step's AdamW)
static ZeroArgs minibatch_zero_args(const Dims& D, const PpoWorkspace& ws, float* grads, double* metrics, int parts) {
    const FlatOffsets FA = make_flat_offsets(D.IN, D.H, D.XD, D.TD);
    const FlatOffsets FC = make_flat_offsets(D.SD, D.HC, 1, 0);
    ZeroArgs z = {};
    const size_t actor_acc = (size_t)((const uint8_t*)(ws.gseg + 16 * D.H) - (const uint8_t*)ws.pl2);   // pl2 | pa0 | gseg
    const size_t critic_acc = (size_t)((const uint8_t*)(ws.crow_cnt + 1) - (const uint8_t*)ws.cpl2);
    if (parts == 3) {
        z.p[0] = grads; z.n[0] = (FA.count + FC.count) * sizeof(float);
        z.p[1] = metrics; z.n[1] = 16 * sizeof(double);
        z.p[2] = ws.pl2; z.n[2] = actor_acc;
        z.p[3] = ws.cpl2; z.n[3] = critic_acc;
    } else if (parts == 1 || parts == 4) {
        z.p[0] = grads; z.n[0] = FA.count * sizeof(float);
        z.p[1] = metrics; z.n[1] = sizeof(double);
        z.p[2] = metrics + 2; z.n[2] = 14 * sizeof(double);
        z.p[3] = ws.pl2; z.n[3] = actor_acc;
    } else if (parts == 2) {
        z.p[0] = grads ? grads + FA.count : nullptr; z.n[0] = FC.count * sizeof(float);
        z.p[1] = metrics + 1; z.n[1] = sizeof(double);
        z.p[2] = ws.cpl2; z.n[2] = critic_acc;
    }
    return z;
}

extern "C" int dppo_ppo_clear_ranges(const dppo_dims* d, int precision, int batch_rows, void* workspace,
                                     double* metrics, int part, void** ptrs, size_t* bytes, int* count) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(workspace && metrics && ptrs && bytes && count && batch_rows > 0, "dppo_ppo_clear_ranges: bad arguments");
    DPPO_CHECK(part == 1 || part == 2 || part == 3 || part == 4, "dppo_ppo_clear_ranges: part must be 1, 2, 3 or 4");
    const PpoWorkspace ws = make_ppo_workspace(D, precision, batch_rows, (uint8_t*)workspace);
    const ZeroArgs z = minibatch_zero_args(D, ws, nullptr, metrics, part);
    int n = 0;
    for (int r = 1; r < 4; ++r)
        if (z.p[r]) { ptrs[n] = z.p[r]; bytes[n] = z.n[r]; ++n; }
    *count = n;
    return DPPO_OK;
}

// parts: 3 = the whole minibatch (critic on the internal side stream); 1 = the actor's half only,
// 2 = the critic's half only, each on the caller's stream (the caller overlaps them; see
// dppo_ppo_minibatch_part in include/dppo.h)
static int ppo_minibatch_impl(const dppo_dims* d, int precision, const dppo_ppo_hparams* hp,
                              const void* packed_ft, const void* packed_critic, const float* actor_params,
                              const float* sched, const float* obs, const float* chains, const float* lp_old_mean,
                              const float* advantages, const float* returns, int64_t total, uint64_t perm_seed,
                              int epoch, int64_t start, int rows, const int64_t* row_index, const double* adv_stats,
                              void* workspace, float* grads, double* metrics, void* stream, int parts) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(hp && packed_ft && packed_critic && actor_params && sched && obs && chains && lp_old_mean && advantages &&
               returns && workspace && grads && metrics, "dppo_ppo_minibatch: null pointer");
    DPPO_CHECK(total > 0 && total % D.KF == 0, "dppo_ppo_minibatch: total must be a positive multiple of K'");
    DPPO_CHECK(rows > 0 && start >= 0, "dppo_ppo_minibatch: bad rows/start");
    DPPO_CHECK(hp->global_rows > 0, "dppo_ppo_minibatch: global_rows must be > 0");
    DPPO_CHECK(D.KF <= 16, "dppo_ppo_minibatch: ft_denoising_steps > 16 unsupported (bucket sums)");
    hipStream_t s = (hipStream_t)stream;
    const PpoWorkspace ws = make_ppo_workspace(D, precision, rows, (uint8_t*)workspace);
    DPPO_CHECK(ws.total < ((size_t)1 << 31), "dppo_ppo_minibatch: workspace for %d rows exceeds 2 GiB", rows);
    const FlatOffsets FA = make_flat_offsets(D.IN, D.H, D.XD, D.TD);
    const FlatOffsets FC = make_flat_offsets(D.SD, D.HC, 1, 0);
    float* ga = grads;
    float* gc = grads + FA.count;
    DPPO_CHECK(parts >= 1 && parts <= 5, "dppo_ppo_minibatch: bad part %d", parts);
    DPPO_CHECK(parts == 3 || adv_stats || parts == 2 || parts == 5,
               "dppo_ppo_minibatch_part: the actor half needs adv_stats");
    DPPO_CHECK((hp->flags & ~(DPPO_PPO_L2_DEFERRED | DPPO_PPO_LEARN_ETA | DPPO_PPO_PRECLEARED)) == 0,
               "dppo_ppo_minibatch: unknown flags 0x%x", hp->flags);
    // one launch zeroes the atomically accumulated outputs of the half (or whole) being run
    // (minibatch_zero_args) unless the caller's optimizer step already did (DPPO_PPO_PRECLEARED)
    const ZeroArgs z = minibatch_zero_args(D, ws, grads, metrics, parts);
    // few workgroups: the split update runs this while the other stream's row tiles hold most CUs,
    // and a 256-block grid waited ~25 us for slots
    // part 5 continues the actor half whose part 4 zeroed its outputs
    if (parts != 5 && !(hp->flags & DPPO_PPO_PRECLEARED)) {
        DppoKtScope kt(KT_ZERO, s);
        hipLaunchKernelGGL(zero_kernel, dim3(16), dim3(256), 0, s, z);
        DPPO_HIP(hipGetLastError());
    }
    DPPO_CHECK((uint64_t)total < ((uint64_t)1 << 32), "dppo_ppo_minibatch: %lld samples x steps exceed 2^32",
               (long long)total);
    const FeistelKey fk = feistel_key((uint64_t)total, perm_seed, epoch);
    const double* stats = adv_stats;
    if (!stats && parts != 2 && parts != 5) {
        const int blocks = dppo_cdiv(rows, 256) < 512 ? dppo_cdiv(rows, 256) : 512;
        hipLaunchKernelGGL(adv_stats_kernel, dim3(blocks), dim3(256), 0, s, advantages, fk, D.KF, start, rows,
                           row_index, ws.stats);
        DPPO_HIP(hipGetLastError());
        stats = ws.stats;
    }
    LossHP lh;
    lh.gamma_denoising = hp->gamma_denoising; lh.clip_coef = hp->clip_ploss_coef;
    lh.clip_coef_base = hp->clip_ploss_coef_base; lh.clip_coef_rate = hp->clip_ploss_coef_rate;
    lh.min_lp_std = hp->min_logprob_std; lh.vf_coef = hp->vf_coef; lh.norm_adv = hp->norm_adv;
    lh.reward_horizon = hp->reward_horizon;
    // fp16: the backward images carry GRAD_SCALE x the gradient (fp16 range); dW divides it out
    const float gscale = dppo_grad_scale_rows(precision, hp->global_rows);
    lh.grad_scale = hp->loss_scale / (float)hp->global_rows * gscale;
    lh.eta_unscale = (hp->flags & DPPO_PPO_LEARN_ETA) ? 1.f / gscale : 0.f;
    lh.clip_vloss = hp->clip_vloss_coef > 0.f && hp->old_values ? hp->clip_vloss_coef : 0.f;
    lh.old_values = lh.clip_vloss > 0.f ? hp->old_values : nullptr;
    // the actor's l2 gradient left factored in its own grads region (include/dppo.h)
    const bool l2_def = (hp->flags & DPPO_PPO_L2_DEFERRED) != 0;

    ActorArgs aa = {};
    aa.packed = (const uint8_t*)packed_ft;
    aa.L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    aa.sched = sched; aa.obs = obs; aa.chains = chains;
    aa.XD = D.XD; aa.SD = D.SD; aa.TD = D.TD; aa.IN = D.IN; aa.H = D.H; aa.KF = D.KF; aa.Da = D.Da; aa.TS = D.TS;
    aa.mode = ROWS_TRAIN; aa.nrows = rows; aa.fk = fk; aa.start = start; aa.row_index = row_index;
    aa.lp_old = lp_old_mean; aa.adv = advantages; aa.adv_stats = stats; aa.hp = lh; aa.ws = ws; aa.metrics = metrics;

    CriticArgs ca = {};
    ca.packed = (const uint8_t*)packed_critic;
    ca.L = make_mlp_layout(D.SD, D.HC, 1, 0, precision);
    ca.obs = obs; ca.SD = D.SD; ca.HC = D.HC; ca.KF = D.KF; ca.mode = ROWS_TRAIN; ca.nrows = rows;
    ca.fk = fk; ca.start = start; ca.row_index = row_index; ca.returns = returns; ca.hp = lh; ca.ws = ws; ca.metrics = metrics;
    // weight-gradient problems of one network, launched as one grouped dW kernel on stream st.
    // m-chunks: about one workgroup per CU (the ring takes 132 KB of LDS) in a single round.
    const int tk = DW_TK;
    const int* crit_rows_dev = nullptr;
    auto launch_grads = [&](bool actor, hipStream_t st) -> int {
        DWArgs w = {};
        int all_tiles = 0;
        if (!actor) w.rows_dev = crit_rows_dev;
        const size_t span = ws.ldm;
        // the critic's dW runs beside the actor's dW tail: its smaller ring (WK = 128, 3 slots) leaves the
        // CU room for the time-MLP backward's workgroup
        const int wk = actor ? tk : 0, tke = wk ? wk : 128;
        auto add = [&](const void* XT, int Kx, const void* DT, int N, float* G, int extra, float* Gx) {
            all_tiles += dppo_cdiv(Kx, tke) * dppo_cdiv(N, DW_TN);
            DWProb& p = w.p[w.nprob];
            p.XT = XT; p.DT = DT; p.G = G; p.Gx = Gx; p.Kx = Kx; p.N = N; p.extra = extra;
            p.ktiles = dppo_cdiv(Kx, tke); p.ntiles = dppo_cdiv(N, DW_TN);
            w.tile_start[w.nprob + 1] = w.tile_start[w.nprob] + p.ktiles * p.ntiles;
            w.nprob++;
        };
        if (actor) {
            add(ws.a0T, D.IN, ws.dh1T, D.H, ga + FA.in_w, EXTRA_ONEHOT, ws.gseg);
            add(ws.u1T, D.H, ws.dh2T, D.H, ga + FA.l1_w, EXTRA_ONES, ga + FA.l1_b);
            add(ws.u2T, D.H, ws.dyT, D.XD, l2_def ? ga + FA.l2_w : ws.pl2, EXTRA_NONE, nullptr);   // l2 through the out layer
            add(ws.a0T, D.IN, ws.dyT, D.XD, ws.pa0, EXTRA_ONES, ga + FA.out_b);   // out through the fold (out_back)
        } else {
            add(ws.csT, D.SD, ws.cdh1T, D.HC, gc + FC.in_w, EXTRA_ONES, gc + FC.in_b);
            add(ws.cu1T, D.HC, ws.cdh2T, D.HC, gc + FC.l1_w, EXTRA_ONES, gc + FC.l1_b);
            add(ws.cu2T, D.HC, ws.cdvT, 1, ws.cpl2, EXTRA_NONE, nullptr);
            add(ws.ch3T, D.HC, ws.cdvT, 1, gc + FC.out_w, EXTRA_ONES, gc + FC.out_b);
        }
        w.ldm = ws.ldm;
        w.seg = ws.seg;
        w.out_scale = 1.f / gscale;
        const int tiles = all_tiles;
        // about one workgroup per CU, but no chunk under 768 rows: at small minibatches (6,250 rows,
        // an 8-GPU rank's share) thinner chunks cost more in partial-tile atomics than they gain
        // in parallelism (0.177 -> 0.154 ms per minibatch, tools/ab_small_mb2.sh)
        int nch = dw_device_cus() / tiles;
        if (nch > (int)(span / 768)) nch = (int)(span / 768);
        const int max_ch = (int)(span / 64);
        if (nch > max_ch) nch = max_ch;
        if (nch < 1) nch = 1;
        w.mchunk = (int)(dppo_cdiv((int)span, nch * 64) * 64);
        w.nchunks = dppo_cdiv((int)span, w.mchunk);
        DppoKtScope kt(actor ? KT_DW_ACTOR : KT_DW_CRITIC, st);
        return precision == DPPO_BF16 ? launch_dw<PolicyBF16>(w, wk, st)
             : precision == DPPO_F16  ? launch_dw<PolicyF16>(w, wk, st) : launch_dw<PolicyF32>(w, wk, st);
    };

    // the critic's distinct samples (sample-weighted value loss, crit_rows_kernel), on the stream
    // the critic's half runs on
    uint32_t* crit_cnt = nullptr;
    auto critic_rows = [&](hipStream_t st) -> int {
        if (!crit_dedup()) return DPPO_OK;
        const int64_t nsamp = total / D.KF;
        { const int rc_ = crit_count_scratch(nsamp, st, &crit_cnt); if (rc_) return rc_; }
        const int blocks = dppo_cdiv(rows, 256) < 512 ? dppo_cdiv(rows, 256) : 512;
        DppoKtScope kt(KT_CRIT_ROWS, st);
        hipLaunchKernelGGL(crit_rows_kernel, dim3(blocks), dim3(256), 0, st, row_index, start, rows, fk, D.KF, crit_cnt,
                           ws.crow_n, ws.crow_cnt);
        DPPO_HIP(hipGetLastError());
        ca.crow_n = ws.crow_n; ca.crow_mult = crit_cnt; ca.crow_cnt = ws.crow_cnt;
        crit_rows_dev = ws.crow_cnt;
        return DPPO_OK;
    };
    auto critic_tail = [&](hipStream_t st) {
        return launch_critic_l2_back(D, precision, ws.cpl2, packed_critic, gc, crit_cnt, ws.crow_n, ws.crow_cnt, st);
    };

    // after the actor's dW: the time-MLP backward, W_out's gradient and (materialised) l2's in one launch.
    // (Forking the time-MLP backward beside the dW (r05, profiles/r05y_tb_fork_ab.txt) and running it
    // inside a one-launch actor step (r06, profiles/r06de_actor_tail_ab.txt) were both measured slower.)
    const float* pl2_src = l2_def ? ga + FA.l2_w : ws.pl2;
    auto actor_grads = [&]() -> int { return launch_grads(true, s); };
    auto actor_tail = [&]() -> int {
        return launch_time_bwd(D, precision, ws.gseg, pl2_src, ws.pa0, packed_ft, actor_params, ga, D.KF, D.TS, s,
                               !l2_def);
    };

    // The critic is independent of the actor: its row tiles and then its weight gradients run on a
    // side stream, filling the CUs the actor's row tiles leave idle (the actor's last partial round)
    // and overlapping the critic's HBM-bound dW with the actor's tiles. Joined before the
    // actor's dW completes the minibatch.
    if (parts == 2) {                                  // the critic's half on the caller's stream
        rc = critic_rows(s);
        if (rc) return rc;
        rc = launch_critic_rowtile(ca, precision, s);
        if (rc) return rc;
        rc = launch_grads(false, s);
        if (rc) return rc;
        return critic_tail(s);
    }
    if (parts == 1 || parts == 4 || parts == 5) {      // the actor's half (or its row tiles / its
        if (parts != 5) {                              // weight gradients) on the caller's stream
            rc = launch_actor_rowtile(aa, precision, s);
            if (rc) return rc;
        }
        if (parts == 4) return DPPO_OK;
        rc = actor_grads();
        if (rc) return rc;
        return actor_tail();
    }
    SideStream* side = side_stream();
    if (side) {
        DPPO_HIP(hipEventRecord(side->fork, s));
        DPPO_HIP(hipStreamWaitEvent(side->stream, side->fork, 0));
        rc = critic_rows(side->stream);
        if (rc) return rc;
        rc = launch_critic_rowtile(ca, precision, side->stream);
        if (rc) return rc;
        rc = launch_grads(false, side->stream);
        if (rc) return rc;
        rc = critic_tail(side->stream);
        if (rc) return rc;
        DPPO_HIP(hipEventRecord(side->join, side->stream));
    }
    if (!side) {
        rc = launch_actor_rowtile(aa, precision, s);
        if (rc) return rc;
        rc = critic_rows(s);
        if (rc) return rc;
        rc = launch_critic_rowtile(ca, precision, s);
        if (rc) return rc;
        rc = launch_grads(false, s);
        if (rc) return rc;
        rc = critic_tail(s);
        if (rc) return rc;
        rc = actor_grads();
        if (rc) return rc;
    } else {
        rc = launch_actor_rowtile(aa, precision, s);
        if (rc) return rc;
        rc = actor_grads();
        if (rc) return rc;
        DPPO_HIP(hipStreamWaitEvent(s, side->join, 0));
    }
    return actor_tail();
}

extern "C" int dppo_ppo_minibatch(const dppo_dims* d, int precision, const dppo_ppo_hparams* hp,
                                  const void* packed_ft, const void* packed_critic, const float* actor_params,
                                  const float* sched, const float* obs, const float* chains, const float* lp_old_mean,
                                  const float* advantages, const float* returns, int64_t total, uint64_t perm_seed,
                                  int epoch, int64_t start, int rows, const int64_t* row_index, const double* adv_stats,
                                  void* workspace, float* grads, double* metrics, void* stream) {
    return ppo_minibatch_impl(d, precision, hp, packed_ft, packed_critic, actor_params, sched, obs, chains, lp_old_mean,
                              advantages, returns, total, perm_seed, epoch, start, rows, row_index, adv_stats, workspace,
                              grads, metrics, stream, 3);
}

extern "C" int dppo_ppo_minibatch_part(const dppo_dims* d, int precision, const dppo_ppo_hparams* hp,
                                       const void* packed_ft, const void* packed_critic, const float* actor_params,
                                       const float* sched, const float* obs, const float* chains,
                                       const float* lp_old_mean, const float* advantages, const float* returns,
                                       int64_t total, uint64_t perm_seed, int epoch, int64_t start, int rows,
                                       const int64_t* row_index, const double* adv_stats, void* workspace,
                                       float* grads, double* metrics, int part, void* stream) {
    DPPO_CHECK(part == 1 || part == 2 || part == 4 || part == 5,
               "dppo_ppo_minibatch_part: part must be 1 (actor), 2 (critic), 4 (actor row tiles) or 5 (actor dW)");
    return ppo_minibatch_impl(d, precision, hp, packed_ft, packed_critic, actor_params, sched, obs, chains, lp_old_mean,
                              advantages, returns, total, perm_seed, epoch, start, rows, row_index, adv_stats, workspace,
                              grads, metrics, stream, part);
}

extern "C" int dppo_materialize_l2(const dppo_dims* d, int precision, const void* packed_actor, float* grads,
                                   void* workspace, int batch_rows, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(packed_actor && grads && workspace && batch_rows > 0, "dppo_materialize_l2: bad arguments");
    hipStream_t s = (hipStream_t)stream;
    const PpoWorkspace ws = make_ppo_workspace(D, precision, batch_rows, (uint8_t*)workspace);
    const FlatOffsets FA = make_flat_offsets(D.IN, D.H, D.XD, D.TD);
    DPPO_HIP(hipMemcpyAsync(ws.pl2, grads + FA.l2_w, sizeof(float) * (size_t)D.H * D.XD, hipMemcpyDeviceToDevice, s));
    const MlpLayout L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    L2Back l2b = {ws.pl2, grads + FA.out_b, (const uint8_t*)packed_actor + L.off[SEG_W_OUT], grads + FA.l2_w,
                  grads + FA.l2_b, D.H, D.XD, precision, nullptr, nullptr, nullptr};
    DPPO_CHECK(D.XD <= L2B_MAXN, "l2_back: action horizon x dim %d > %d", D.XD, L2B_MAXN);
    launch_l2_back(precision, (unsigned)dppo_cdiv(D.H, L2B_ROWS), s, l2b, dppo_cdiv(D.H, L2B_ROWS), OutBack{}, 0);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// ---------------------------------------------------------------------------------------------
// pretraining loss: DiffusionModel.p_losses / q_sample (diffusion.py:179-202)
// ---------------------------------------------------------------------------------------------
// per-t bucket sums of dh1 for t in [0, nb): G[q][n] = sum over rows with seg == q of dh1T[n][row].
// One workgroup per hidden unit n; each wave bins its rows in LDS (nb <= 64), then the waves' bins
// are added in a fixed order (no global atomics: one writer per (q, n)).
template <class AT>
__global__ __launch_bounds__(256) void seg_reduce_kernel(const AT* __restrict__ dT, const int8_t* __restrict__ seg,
                                                         size_t ldm, int nb, float* __restrict__ G, int H, float scale) {
    __shared__ float bins[4][64];
    const int n = blockIdx.x, tid = threadIdx.x, wave = tid >> 6;
    for (int i = tid; i < 4 * 64; i += 256) (&bins[0][0])[i] = 0.f;
    __syncthreads();
    const AT* row = dT + (size_t)n * ldm;
#pragma unroll 4
    for (size_t r = tid; r < ldm; r += 256) {
        const int q = seg[r];
        if (q >= 0 && q < nb) atomicAdd(&bins[wave][q], (float)row[r]);
    }
    __syncthreads();
    if (tid < nb) G[(size_t)tid * H + n] = ((bins[0][tid] + bins[1][tid]) + (bins[2][tid] + bins[3][tid])) * scale;
}

extern "C" int dppo_pretrain_minibatch(const dppo_dims* d, int precision, const void* packed_actor, const float* actor_params,
                                       const float* sched, const float* qsched, const float* x_start, const float* cond,
                                       const int32_t* t, const float* noise, int rows, int64_t global_rows,
                                       float loss_scale, void* workspace, float* grads, double* metrics, void* stream) {
    Dims D;
    int rc = dppo_check_dims(d, &D);
    if (rc) return rc;
    DPPO_CHECK(dppo_prec_ok(precision), "bad precision %d", precision);
    DPPO_CHECK(packed_actor && actor_params && sched && qsched && x_start && cond && t && noise && workspace && grads &&
               metrics, "dppo_pretrain_minibatch: null pointer");
    DPPO_CHECK(rows > 0 && global_rows >= rows, "dppo_pretrain_minibatch: bad rows / global_rows");
    DPPO_CHECK(D.TS == 1, "dppo_pretrain_minibatch: the time-embedding table must be unstrided (time_stride 1)");
    DPPO_CHECK(D.K <= 64, "dppo_pretrain_minibatch: denoising_steps > 64 unsupported (bucket sums)");
    hipStream_t s = (hipStream_t)stream;
    const PpoWorkspace ws = make_ppo_workspace(D, precision, rows, (uint8_t*)workspace);
    DPPO_CHECK(ws.total < ((size_t)1 << 31), "dppo_pretrain_minibatch: workspace for %d rows exceeds 2 GiB", rows);
    const FlatOffsets FA = make_flat_offsets(D.IN, D.H, D.XD, D.TD);
    float* ga = grads;
    ZeroArgs z = {};
    z.p[0] = grads; z.n[0] = FA.count * sizeof(float);
    z.p[1] = metrics; z.n[1] = 16 * sizeof(double);
    z.p[2] = ws.pl2; z.n[2] = (size_t)((const uint8_t*)ws.gseg - (const uint8_t*)ws.pl2);   // pl2 | pa0
    hipLaunchKernelGGL(zero_kernel, dim3(256), dim3(256), 0, s, z);
    DPPO_HIP(hipGetLastError());

    ActorArgs aa = {};
    aa.packed = (const uint8_t*)packed_actor;
    aa.L = make_mlp_layout(D.IN, D.H, D.XD, D.TD, precision, D.K);
    aa.sched = sched; aa.obs = cond; aa.chains = x_start;
    aa.XD = D.XD; aa.SD = D.SD; aa.TD = D.TD; aa.IN = D.IN; aa.H = D.H; aa.KF = D.K; aa.Da = D.Da; aa.TS = 1;
    aa.mode = ROWS_PRETRAIN; aa.nrows = rows; aa.ws = ws; aa.metrics = metrics;
    aa.tsteps = t; aa.noise = noise; aa.qsched = qsched;
    // loss = mean over global_rows * XD elements of (eps - noise)^2 (diffusion.py:192)
    const float gscale = dppo_grad_scale_rows(precision, global_rows);
    aa.pre_scale = 2.f * loss_scale / ((float)global_rows * (float)D.XD) * gscale;
    rc = launch_actor_rowtile(aa, precision, s);
    if (rc) return rc;

    const int tk = DW_TK;
    DWArgs w = {};
    auto add = [&](const void* XT, int Kx, const void* DT, int N, float* G, int extra, float* Gx) {
        DWProb& p = w.p[w.nprob];
        p.XT = XT; p.DT = DT; p.G = G; p.Gx = Gx; p.Kx = Kx; p.N = N; p.extra = extra;
        p.ktiles = dppo_cdiv(Kx, tk); p.ntiles = dppo_cdiv(N, DW_TN);
        w.tile_start[w.nprob + 1] = w.tile_start[w.nprob] + p.ktiles * p.ntiles;
        w.nprob++;
    };
    // the in-layer's bias and time-MLP gradients come from K bucket sums (seg_reduce + time_bwd)
    add(ws.a0T, D.IN, ws.dh1T, D.H, ga + FA.in_w, EXTRA_NONE, nullptr);
    add(ws.u1T, D.H, ws.dh2T, D.H, ga + FA.l1_w, EXTRA_ONES, ga + FA.l1_b);
    add(ws.u2T, D.H, ws.dyT, D.XD, ws.pl2, EXTRA_NONE, nullptr);   // l2 through the out layer
    add(ws.a0T, D.IN, ws.dyT, D.XD, ws.pa0, EXTRA_ONES, ga + FA.out_b);   // out through the fold (out_back)
    w.ldm = ws.ldm;
    w.seg = ws.seg;
    w.out_scale = 1.f / gscale;
    const int tiles = w.tile_start[w.nprob];
    int nch = dw_device_cus() / tiles;
    const int max_ch = (int)(ws.ldm / 64);
    if (nch > max_ch) nch = max_ch;
    if (nch < 1) nch = 1;
    w.mchunk = (int)(dppo_cdiv((int)ws.ldm, nch * 64) * 64);
    w.nchunks = dppo_cdiv((int)ws.ldm, w.mchunk);
    rc = precision == DPPO_BF16 ? launch_dw<PolicyBF16>(w, tk, s)
       : precision == DPPO_F16  ? launch_dw<PolicyF16>(w, tk, s) : launch_dw<PolicyF32>(w, tk, s);
    if (rc) return rc;
    const float inv = 1.f / gscale;
    if (precision == DPPO_BF16)
        hipLaunchKernelGGL(seg_reduce_kernel<__bf16>, dim3(D.H), dim3(256), 0, s, (const __bf16*)ws.dh1T, ws.seg, ws.ldm,
                           D.K, ws.gseg, D.H, inv);
    else if (precision == DPPO_F16)
        hipLaunchKernelGGL(seg_reduce_kernel<_Float16>, dim3(D.H), dim3(256), 0, s, (const _Float16*)ws.dh1T, ws.seg,
                           ws.ldm, D.K, ws.gseg, D.H, inv);
    else
        hipLaunchKernelGGL(seg_reduce_kernel<float>, dim3(D.H), dim3(256), 0, s, (const float*)ws.dh1T, ws.seg, ws.ldm,
                           D.K, ws.gseg, D.H, inv);
    DPPO_HIP(hipGetLastError());
    return launch_time_bwd(D, precision, ws.gseg, ws.pl2, ws.pa0, packed_actor, actor_params, ga, D.K, 1, s);
}
