// dppo_ppo.h — argument blocks and workspace layout of the PPO-update kernels.
#pragma once
#include "dppo_common.cuh"
#include "dppo_internal.h"

// feature-major ("transposed") activation / gradient images written by the row-tile kernels and
// consumed by the split-K weight-gradient kernel: X^T[f][ldm], ldm = rows rounded up to 64.
struct PpoWorkspace {
    uint8_t* base;    // start of the workspace (buffer-resource base of the image stores)
    size_t ldm;
    // actor (no dh3 image: l2's weight gradient is formed through the out layer, see pl2; no h3 image:
    // the folded row tile never forms h3, see pa0)
    void *a0T, *u1T, *u2T, *dyT, *dh2T, *dh1T;
    // critic
    void *csT, *cu1T, *cu2T, *ch3T, *cdvT, *cdh2T, *cdh1T;
    int8_t* seg;      // [ldm] t of each row (bucket id for the one-hot bias/temb sums), -1 invalid
    // l2's weight gradient through the linear out layer: dh3 = dy W_out^T, so
    //   dW_l2 = u2^T dh3 = (u2^T dy) W_out^T,  db_l2 = (1^T dy) W_out^T = db_out W_out^T
    // pl2 = u2^T dy [H][XD] (actor) and cpl2 = cu2^T dv [HC] (critic) come from the dW GEMM (K = rows),
    // the H x H products from l2_back_kernel. Each is followed by the buffer zeroed with it: pl2 |
    // gseg, cpl2 | stats
    float* pl2;
    // W_out's weight gradient through the folded forward (h3 = u2 W_l2 + a0 W_in + b_l2 + b_in):
    //   dW_out = W_l2^T pl2 + W_in^T pa0 + (b_l2 + b_in) db_out,  pa0 = a0^T dy [IN][XD] (dW GEMM),
    // formed by the out_back groups after the dW (update.hip); zeroed with pl2 | pa0 | gseg
    float* pa0;
    float* gseg;      // [64][H] per-t sums of dh1 (actor in-layer; 16 buckets in PPO, K in pretraining)
    float* cpl2;
    double* stats;    // [4] adv {count, sum, sumsq}
    // the critic's distinct samples of a minibatch (sample-weighted value loss, ppo_minibatch_impl):
    // crow_n [ldm] sample indices in arrival order, crow_cnt [1] how many (zeroed with cpl2 | stats;
    // the multiplicities stay in the per-stream count scratch, crit_rows_kernel)
    int* crow_n;
    int* crow_cnt;
    size_t total;
};

inline PpoWorkspace make_ppo_workspace(const Dims& D, int precision, int rows, uint8_t* base) {
    PpoWorkspace w;
    w.base = base;
    const size_t es = dppo_prec_2b(precision) ? 2 : 4;
    w.ldm = (size_t)dppo_cdiv(rows > 0 ? rows : 1, 64) * 64;
    size_t o = 0;
    auto take = [&](size_t feats) -> void* {
        void* p = base ? (void*)(base + o) : nullptr;
        o = dppo_align256(o + feats * w.ldm * es);
        return p;
    };
    w.a0T = take(D.IN); w.u1T = take(D.H); w.u2T = take(D.H);
    w.dyT = take(D.XD); w.dh2T = take(D.H); w.dh1T = take(D.H);
    w.csT = take(D.SD); w.cu1T = take(D.HC); w.cu2T = take(D.HC); w.ch3T = take(D.HC);
    w.cdvT = take(1); w.cdh2T = take(D.HC); w.cdh1T = take(D.HC);
    w.seg = base ? (int8_t*)(base + o) : nullptr; o = dppo_align256(o + w.ldm);
    w.pl2 = base ? (float*)(base + o) : nullptr; o = dppo_align256(o + 4 * (size_t)D.H * D.XD);
    w.pa0 = base ? (float*)(base + o) : nullptr; o = dppo_align256(o + 4 * (size_t)D.IN * D.XD);
    w.gseg = base ? (float*)(base + o) : nullptr; o = dppo_align256(o + 4 * 64 * (size_t)D.H);
    w.cpl2 = base ? (float*)(base + o) : nullptr; o = dppo_align256(o + 4 * (size_t)D.HC);
    w.stats = base ? (double*)(base + o) : nullptr; o += 8 * 4;
    w.crow_cnt = base ? (int*)(base + o) : nullptr; o = dppo_align256(o + 4);
    w.crow_n = base ? (int*)(base + o) : nullptr; o = dppo_align256(o + 4 * w.ldm);
    w.total = o;
    return w;
}

// byte offset of an image inside the workspace (< 2 GiB: checked by dppo_ppo_minibatch)
__host__ __device__ inline uint32_t ws_off(const PpoWorkspace& w, const void* img) {
    return (uint32_t)((const uint8_t*)img - w.base);
}

// per-row source of a row-tile launch
// ROWS_PRETRAIN: the pretraining loss p_losses (diffusion.py:179-202) through the TRAIN row tile:
// row r is sample r, t and noise come with it, KF holds K (every t is a bucket)
enum { ROWS_LOGPROB = 0, ROWS_TRAIN = 1, ROWS_VALUE = 2, ROWS_PRETRAIN = 3 };

struct LossHP {
    float gamma_denoising, clip_coef, clip_coef_base, clip_coef_rate, min_lp_std, vf_coef;
    int norm_adv, reward_horizon;
    float grad_scale;     // loss_scale / global_rows
    float eta_unscale;    // learnable DDIM eta (DPPO_PPO_LEARN_ETA): 1 / the fp16 seed scale, else 0
    float clip_vloss;     // > 0: the clipped value loss against old_values (diffusion_ppo.py:110-116)
    const float* old_values;
};

struct ActorArgs {
    const uint8_t* packed;
    MlpLayout L;
    const float* sched;
    const float* obs;      // [nsamp][SD]
    const float* chains;   // [nsamp][KF+1][XD]
    int XD, SD, TD, IN, H, KF, Da, mode;
    int TS;                // time stride: row r of the time embeddings is t_emb(r TS)
    int64_t nrows;         // logprob: nsamp*KF; train: rows
    // logprob outputs
    float* lp_elem;
    float* lp_mean;
    // train
    FeistelKey fk;
    int64_t start;
    const int64_t* row_index;
    const float* lp_old;   // [nsamp][KF]
    const float* adv;      // [nsamp]
    const double* adv_stats;
    LossHP hp;
    PpoWorkspace ws;
    double* metrics;
    // pretrain (ROWS_PRETRAIN): chains = x_start [rows][XD], obs = cond [rows][SD]
    const int* tsteps;     // [rows] t in [0, K)
    const float* noise;    // [rows][XD]
    const float* qsched;   // [K][2] sqrt(alphas_cumprod), sqrt(1 - alphas_cumprod)
    float pre_scale;       // d loss / d eps = pre_scale * (eps - noise)
    // tile range of one launch: image rows [row0, row_end); row_end = 0: all rows of the mode
    int64_t row0, row_end;
};

struct CriticArgs {
    const uint8_t* packed;
    MlpLayout L;
    const float* obs;
    int SD, HC, KF, mode;
    int64_t nrows;
    float* values;        // value mode
    FeistelKey fk;
    int64_t start;
    const int64_t* row_index;
    const float* returns;
    LossHP hp;
    PpoWorkspace ws;
    double* metrics;
    // TRAIN with crow_n != null: row r is distinct sample n = crow_n[r] with weight crow_mult[n] (its
    // multiplicity in the minibatch), *crow_cnt rows (device-side count); the value loss and its
    // gradient are the per-row ones summed over the copies
    const int* crow_n;
    const uint32_t* crow_mult;
    const int* crow_cnt;
};

int launch_actor_rowtile(const ActorArgs& a, int precision, hipStream_t s);
int launch_critic_rowtile(const CriticArgs& a, int precision, hipStream_t s);
