// dppo_layout.h — host+device description of the packed (MFMA fragment-ordered) weight images.
//
// A residual MLP (model/common/mlp.py:95-206: in-Dense, one pre-activation two-Dense block,
// out-Dense) is stored as segments, each 256-B aligned:
//   TIME   fp32 time MLP (actor only): w1[TD,2TD] b1[2TD] w2[2TD,TD] b2[TD]
//   W_IN   packed fwd  [K=in_dim][N=H]      B_IN  fp32 [H]
//   W_L1   packed fwd  [H][H]               B_L1  fp32 [H]
//   W_L2   packed fwd  [H][H]               B_L2  fp32 [H]
//   W_OUT  packed fwd  [H][out]             B_OUT fp32 [16*ceil(out/16)] (zero padded)
//   T_OUT  packed bwd  W_out^T as [K=out][N=H]
//   T_L2   packed bwd  W_l2^T  as [K=H][N=H]
//   T_L1   packed bwd  W_l1^T  as [K=H][N=H]
//   TEMB   fp32 [K][TD] time embeddings t_emb(t) for t = 0..K-1 (actor only; derived from TIME at
//          pack time, so no kernel re-evaluates the time MLP per launch)
// and, for an actor, three segments derived for the split sampler (sampler_split.hip), whose
// in-Dense then only multiplies the per-step inputs:
//   W_XS   packed fwd  W_in rows [x ; state] (in-Dense input rows 0..XD-1 and XD+TD..in_dim-1)
//   TIN    fp32 [K][H] b_in + W_in[temb rows]^T t_emb(t): the in-Dense's time part per t (2-byte
//          precisions: operands rounded as the kernels round them, fp32 sums)
//   B_OUT2 fp32 [16*ceil(out/16)] b_out + W_out^T b_l2: the l2 bias folded through the out-Dense
//          (the residual block is linear from the l2 product to the out-Dense, mlp.py:186-206)
//   FOLD   [nt_h][nt_out] 1 KiB fragments of M = rnd(W_l2) rnd(W_out) (fp32 product, [H][out]): the
//          l2 layer folded into the out-Dense for the same reason, so the sampler's eps is
//          W_out^T h1 + M^T relu(h2) + B_OUT2 and l2 never runs as a GEMM. Lane l of fragment
//          (T, n) holds, for out o = 16n + (l&15) and features f = 16T + 4(l>>4) + e, e < 4:
//          k-slots 0-3 = hi(M[f][o]), 4-7 = lo(M[f][o]) (2-byte hi/lo pair: the product's fp32
//          value to ~16 bits), for a B operand that repeats the 4 activations in both halves
//   ROUT   the same geometry with both halves = rnd(W_out[f][o]) (the residual h1 term, whose B
//          operand is h1's hi/lo pair)
// and, for an actor, the same fold for the row tiles (rowtile.hip), whose forward then runs no l2
// GEMM (eps = relu(h2) M + a0 M0 + RT_BOUT) and whose backward forms d relu(h2) = dy M^T (no dh3 W_l2^T
// GEMM). NHL = 2 hi/lo copies for 2-byte operands (the fp32 product to ~16 bits), 1 for fp32:
//   RT_FOLD    NHL packed fwd [K=H][N=out] matrices: M = rnd(W_l2) rnd(W_out) (hi, then lo)
//   RT_FOLD0   NHL packed fwd [K=in_dim][N=out]: M0 = rnd(W_in) rnd(W_out) (the residual h1 through the
//              out-Dense, from the in-Dense's input)
//   RT_TFOLD   packed bwd [K=ks_out_t*KG][N=H]: element (k, f) = hi(M[f][k]) for k < out, and (2-byte)
//              lo(M[f][k - LOK]) for LOK <= k < LOK + out, LOK = ks_out_t*KG/2, against a dy tile whose
//              columns [LOK, LOK + out) repeat dy: one GEMM of the dy tile's width gives both halves
//   RT_BOUT    fp32 [16*ceil(out/16)] b_out + sum_h (b_in[h] + b_l2[h]) rnd(W_out[h][o])
// A packed matrix [K][N] is ceil(N/16) n-tiles x KS k-steps x 64 lanes x 16 B, with
// KS = ceil(K / KG) rounded up to EVEN (the weight stream runs in k-step pairs), KG = 32 (bf16)
// or 16 (fp32). Lane l of (ntile, ks) holds, for e < EPL,
//   W[ks*KG + (l>>4)*EPL + e][ntile*16 + (l&15)]   (zero outside [K][N]).
#pragma once
#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define DPPO_HD __host__ __device__
#else
#define DPPO_HD
#endif

enum MlpSeg { SEG_TIME = 0, SEG_W_IN, SEG_B_IN, SEG_W_L1, SEG_B_L1, SEG_W_L2, SEG_B_L2, SEG_W_OUT, SEG_B_OUT,
              SEG_T_OUT, SEG_T_L2, SEG_T_L1, SEG_TEMB, SEG_W_XS, SEG_TIN, SEG_B_OUT2,
              SEG_FOLD, SEG_ROUT, SEG_RT_FOLD, SEG_RT_FOLD0, SEG_RT_TFOLD, SEG_RT_BOUT, SEG_COUNT };

struct MlpLayout {
    int in_dim, hidden, out_dim, time_dim, precision, temb_steps;
    int KG;                 // 32 bf16 / 16 fp32
    int ks_in, ks_h, ks_out_t;   // k-steps: in layer, hidden layers, transposed out (K = out_dim)
    int nt_h, nt_out;       // n-tiles: hidden, out
    size_t off[SEG_COUNT];
    size_t total;
};

DPPO_HD inline size_t dppo_align256(size_t x) { return (x + 255) & ~(size_t)255; }
DPPO_HD inline size_t dppo_align16(size_t x) { return (x + 15) & ~(size_t)15; }
DPPO_HD inline int dppo_cdiv(int a, int b) { return (a + b - 1) / b; }
DPPO_HD inline int packed_ksteps(int K, int KG) { return (dppo_cdiv(K, KG) + 1) & ~1; }
DPPO_HD inline size_t packed_matrix_bytes(int K, int N, int KG) {
    return (size_t)dppo_cdiv(N, 16) * (size_t)packed_ksteps(K, KG) * 64 * 16;
}

// hi/lo copies of the row tiles' fold fragments (dppo_layout.h RT_*), and the k offset of the lo half
// of RT_TFOLD (2-byte operands: half the transposed out-layer's k extent)
DPPO_HD inline int rt_fold_copies(int precision) { return (precision == 1 || precision == 2) ? 2 : 1; }
DPPO_HD inline int rt_tfold_lok(int ks_out_t, int KG) { return ks_out_t * KG / 2; }

DPPO_HD inline MlpLayout make_mlp_layout(int in_dim, int hidden, int out_dim, int time_dim, int precision,
                                         int temb_steps = 0) {
    MlpLayout L;
    L.in_dim = in_dim; L.hidden = hidden; L.out_dim = out_dim; L.time_dim = time_dim; L.precision = precision;
    L.temb_steps = time_dim > 0 ? temb_steps : 0;
    L.KG = (precision == 1 || precision == 2) ? 32 : 16;     // bf16 / fp16: 32; fp32: 16
    L.ks_in = packed_ksteps(in_dim, L.KG);
    L.ks_h = packed_ksteps(hidden, L.KG);
    L.ks_out_t = packed_ksteps(out_dim, L.KG);
    L.nt_h = dppo_cdiv(hidden, 16);
    L.nt_out = dppo_cdiv(out_dim, 16);
    size_t o = 0;
    const size_t tsz = time_dim > 0 ? (size_t)4 * (time_dim * 2 * time_dim + 2 * time_dim + 2 * time_dim * time_dim + time_dim) : 0;
    L.off[SEG_TIME] = o; o = dppo_align256(o + tsz);
    L.off[SEG_W_IN] = o; o = dppo_align256(o + packed_matrix_bytes(in_dim, hidden, L.KG));
    L.off[SEG_B_IN] = o; o = dppo_align256(o + (size_t)4 * hidden);
    L.off[SEG_W_L1] = o; o = dppo_align256(o + packed_matrix_bytes(hidden, hidden, L.KG));
    L.off[SEG_B_L1] = o; o = dppo_align256(o + (size_t)4 * hidden);
    L.off[SEG_W_L2] = o; o = dppo_align256(o + packed_matrix_bytes(hidden, hidden, L.KG));
    L.off[SEG_B_L2] = o; o = dppo_align256(o + (size_t)4 * hidden);
    L.off[SEG_W_OUT] = o; o = dppo_align256(o + packed_matrix_bytes(hidden, out_dim, L.KG));
    L.off[SEG_B_OUT] = o; o = dppo_align256(o + (size_t)4 * 16 * L.nt_out);
    L.off[SEG_T_OUT] = o; o = dppo_align256(o + packed_matrix_bytes(out_dim, hidden, L.KG));
    L.off[SEG_T_L2] = o; o = dppo_align256(o + packed_matrix_bytes(hidden, hidden, L.KG));
    L.off[SEG_T_L1] = o; o = dppo_align256(o + packed_matrix_bytes(hidden, hidden, L.KG));
    L.off[SEG_TEMB] = o; o = dppo_align256(o + (size_t)4 * L.temb_steps * time_dim);
    const int xs_rows = time_dim > 0 ? in_dim - time_dim : 0;     // [x ; state]
    L.off[SEG_W_XS] = o; o = dppo_align256(o + (xs_rows > 0 ? packed_matrix_bytes(xs_rows, hidden, L.KG) : 0));
    L.off[SEG_TIN] = o; o = dppo_align256(o + (size_t)4 * L.temb_steps * hidden);
    L.off[SEG_B_OUT2] = o; o = dppo_align256(o + (time_dim > 0 ? (size_t)4 * 16 * L.nt_out : 0));
    const size_t fold_bytes = time_dim > 0 ? (size_t)L.nt_h * L.nt_out * 1024 : 0;
    L.off[SEG_FOLD] = o; o = dppo_align256(o + fold_bytes);
    L.off[SEG_ROUT] = o; o = dppo_align256(o + fold_bytes);
    const bool rt = time_dim > 0;           // actor: the row tiles' fold
    const int nhl = rt_fold_copies(precision);
    L.off[SEG_RT_FOLD] = o; o = dppo_align256(o + (rt ? nhl * packed_matrix_bytes(hidden, out_dim, L.KG) : 0));
    L.off[SEG_RT_FOLD0] = o; o = dppo_align256(o + (rt ? nhl * packed_matrix_bytes(in_dim, out_dim, L.KG) : 0));
    L.off[SEG_RT_TFOLD] = o;
    o = dppo_align256(o + (rt ? packed_matrix_bytes(L.ks_out_t * L.KG, hidden, L.KG) : 0));
    L.off[SEG_RT_BOUT] = o; o = dppo_align256(o + (rt ? (size_t)4 * 16 * L.nt_out : 0));
    L.total = o;
    return L;
}

// flat fp32 parameter offsets (include/dppo.h layout)
struct FlatOffsets {
    size_t time_w1, time_b1, time_w2, time_b2, in_w, in_b, l1_w, l1_b, l2_w, l2_b, out_w, out_b, count;
};
DPPO_HD inline FlatOffsets make_flat_offsets(int in_dim, int hidden, int out_dim, int time_dim) {
    FlatOffsets f;
    size_t o = 0;
    f.time_w1 = o; o += (size_t)time_dim * 2 * time_dim;
    f.time_b1 = o; o += (size_t)2 * time_dim;
    f.time_w2 = o; o += (size_t)2 * time_dim * time_dim;
    f.time_b2 = o; o += (size_t)time_dim;
    f.in_w = o; o += (size_t)in_dim * hidden;
    f.in_b = o; o += hidden;
    f.l1_w = o; o += (size_t)hidden * hidden;
    f.l1_b = o; o += hidden;
    f.l2_w = o; o += (size_t)hidden * hidden;
    f.l2_b = o; o += hidden;
    f.out_w = o; o += (size_t)hidden * out_dim;
    f.out_b = o; o += out_dim;
    f.count = o;
    return f;
}

// actor: in = XD + TD + SD, out = XD, time_dim = TD; critic: in = SD, out = 1, time_dim = 0
struct ModelDims {
    int XD, SD, TD, H, HC, K, KF, Ta, Da;
};
