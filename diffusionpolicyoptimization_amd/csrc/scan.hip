// scan.hip — a18 RunningRewardScaler (util/reward_scaling.py:13-87) and a19 GAE
// (agent/finetune/train_ppo_diffusion_agent.py:239-263) as wave-level affine-map scans.
//
// Both recurrences are first-order affine: y_t = d_t + c_t * y_{t-/+1}. One wavefront owns one
// env: each lane folds a contiguous chunk of time steps into a map (C, D), the 64 maps are
// composed with a 6-step shuffle scan, and each lane replays its chunk from the scanned carry.
// Arithmetic is fp64 like the reference's NumPy float64 path.
#include "dppo_common.cuh"
#include "dppo_internal.h"

#define SCAN_WAVES 4

// inclusive composition over lanes. forward=true: lane l gets M_l o ... o M_0 (prefix, carry in from
// lower t); forward=false: lane l gets M_l o M_{l+1} o ... o M_63 (suffix, carry from higher t).
__device__ inline void affine_scan(double& C, double& D, int lane, bool forward) {
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const double oc = forward ? __shfl_up(C, off, 64) : __shfl_down(C, off, 64);
        const double od = forward ? __shfl_up(D, off, 64) : __shfl_down(D, off, 64);
        const bool has = forward ? (lane >= off) : (lane + off < 64);
        if (has) {  // (M_self o M_other)(y) = D + C*(od + oc*y)
            D = D + C * od;
            C = C * oc;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// GAE: A_t = delta_t + gamma*lam*nonterm_t * A_{t+1}; R = A + V
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * SCAN_WAVES) void gae_kernel(const double* __restrict__ rew, const float* __restrict__ val,
                                                              const float* __restrict__ last_val, const uint8_t* __restrict__ term,
                                                              int S, int E, double gamma, double lam, double rsc,
                                                              float* __restrict__ adv, float* __restrict__ ret) {
    const int lane = threadIdx.x & 63;
    const int e = blockIdx.x * SCAN_WAVES + (threadIdx.x >> 6);
    if (e >= E) return;
    const int CH = (S + 63) / 64;
    const int t0 = lane * CH, t1 = min(S, t0 + CH);
    auto delta_c = [&](int t, double& dl, double& c) {
        const double nonterm = 1.0 - (double)term[(size_t)t * E + e];
        const double nextv = (t == S - 1) ? (double)last_val[e] : (double)val[(size_t)(t + 1) * E + e];
        dl = rew[(size_t)t * E + e] * rsc + gamma * nextv * nonterm - (double)val[(size_t)t * E + e];
        c = gamma * lam * nonterm;
    };
    // chunk map, processed from t1-1 down to t0: y(t0) = D + C * y(t1)
    double C = 1.0, D = 0.0;
    for (int t = t1 - 1; t >= t0; --t) {
        double dl, c;
        delta_c(t, dl, c);
        D = dl + c * D;
        C = c * C;
    }
    affine_scan(C, D, lane, false);
    // carry into this chunk = y at t1 = scanned D of lane+1 (applied to y_S = 0)
    double carry = __shfl_down(D, 1, 64);
    if (lane == 63) carry = 0.0;
    for (int t = t1 - 1; t >= t0; --t) {
        double dl, c;
        delta_c(t, dl, c);
        carry = dl + c * carry;
        adv[(size_t)t * E + e] = (float)carry;
        ret[(size_t)t * E + e] = (float)(carry + (double)val[(size_t)t * E + e]);
    }
}

// ---------------------------------------------------------------------------------------------
// reward scaler pass 1: rets_t = r_t + (1-first_t)*gamma*rets_{t-1}; per-env Chan moments
// ---------------------------------------------------------------------------------------------
__device__ inline void chan_merge(double& n, double& mean, double& m2, double nb, double meanb, double m2b) {
    if (nb == 0.0) return;
    if (n == 0.0) { n = nb; mean = meanb; m2 = m2b; return; }
    const double tot = n + nb;
    const double delta = meanb - mean;
    mean = mean + delta * nb / tot;
    m2 = m2 + m2b + delta * delta * n * nb / tot;
    n = tot;
}

__global__ __launch_bounds__(64 * SCAN_WAVES) void rets_kernel(const double* __restrict__ rew, const uint8_t* __restrict__ first,
                                                               double* __restrict__ ret_state, double* __restrict__ rets,
                                                               double* __restrict__ env_mom, int S, int E, double gamma) {
    const int lane = threadIdx.x & 63;
    const int e = blockIdx.x * SCAN_WAVES + (threadIdx.x >> 6);
    if (e >= E) return;
    const int CH = (S + 63) / 64;
    const int t0 = lane * CH, t1 = min(S, t0 + CH);
    double C = 1.0, D = 0.0;  // y(t1-1) = D + C * y(t0-1)
    for (int t = t0; t < t1; ++t) {
        const double g = (1.0 - (double)first[(size_t)t * E + e]) * gamma;
        D = rew[(size_t)t * E + e] + g * D;
        C = g * C;
    }
    affine_scan(C, D, lane, true);
    const double y0 = ret_state[e];
    // scanned map of lane l-1 applied to y0 gives the carry into lane l
    double pc = __shfl_up(C, 1, 64), pd = __shfl_up(D, 1, 64);
    double carry = lane == 0 ? y0 : pd + pc * y0;
    double n = 0.0, mean = 0.0, m2 = 0.0;
    for (int t = t0; t < t1; ++t) {
        const double g = (1.0 - (double)first[(size_t)t * E + e]) * gamma;
        carry = rew[(size_t)t * E + e] + g * carry;
        rets[(size_t)t * E + e] = carry;
        n += 1.0;  // Welford
        const double dlt = carry - mean;
        mean += dlt / n;
        m2 += dlt * (carry - mean);
    }
    // last step's ret becomes the carried state (reward_scaling.py:62)
    if (t1 == S && t0 < t1) ret_state[e] = carry;
    // merge moments across the wave
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double on = __shfl_xor(n, off, 64), om = __shfl_xor(mean, off, 64), o2 = __shfl_xor(m2, off, 64);
        chan_merge(n, mean, m2, on, om, o2);
    }
    if (lane == 0) { env_mom[3 * e + 0] = n; env_mom[3 * e + 1] = mean; env_mom[3 * e + 2] = m2; }
}

// merge per-env moments -> moments[3] = {n, mean, M2}; if rms != null also apply the
// RunningMeanStd.update_from_moments (reward_scaling.py:29-39) to rms = {mean, var, count}
__global__ void moments_kernel(const double* __restrict__ env_mom, int E, double* __restrict__ moments, double* __restrict__ rms) {
    __shared__ double sh[3 * 64];
    const int tid = threadIdx.x;
    double n = 0.0, mean = 0.0, m2 = 0.0;
    for (int e = tid; e < E; e += 64) chan_merge(n, mean, m2, env_mom[3 * e], env_mom[3 * e + 1], env_mom[3 * e + 2]);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double on = __shfl_xor(n, off, 64), om = __shfl_xor(mean, off, 64), o2 = __shfl_xor(m2, off, 64);
        chan_merge(n, mean, m2, on, om, o2);
    }
    (void)sh;
    if (tid == 0) {
        moments[0] = n; moments[1] = mean; moments[2] = m2;
        if (rms) {
            const double bm = mean, bv = n > 0 ? m2 / n : 0.0, bc = n;
            const double delta = bm - rms[0];
            const double tot = rms[2] + bc;
            const double new_mean = rms[0] + delta * bc / tot;
            const double M2 = rms[1] * rms[2] + bv * bc + delta * delta * rms[2] * bc / tot;
            rms[0] = new_mean;
            rms[1] = M2 / (tot - 1.0);
            rms[2] = tot;
        }
    }
}

__global__ void scale_apply_kernel(double* __restrict__ rew, const double* __restrict__ rms, int64_t n, double cliprew, double eps) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double s = sqrt(rms[1] + eps);
    double r = rew[i] / s;
    r = r < -cliprew ? -cliprew : (r > cliprew ? cliprew : r);
    rew[i] = r;
}

extern "C" int dppo_gae(const double* reward, const float* values, const float* last_values, const uint8_t* terminated,
                        int S, int E, double gamma, double lam, double reward_scale_const,
                        float* advantages, float* returns, void* stream) {
    DPPO_CHECK(S >= 0 && E >= 0, "dppo_gae: negative size");
    if (S == 0 || E == 0) return DPPO_OK;
    DPPO_CHECK(reward && values && last_values && terminated && advantages && returns, "dppo_gae: null pointer");
    { DppoKtScope kt(KT_GAE, (hipStream_t)stream);
        hipLaunchKernelGGL(gae_kernel, dim3(dppo_cdiv(E, SCAN_WAVES)), dim3(64 * SCAN_WAVES), 0, (hipStream_t)stream,
                           reward, values, last_values, terminated, S, E, gamma, lam, reward_scale_const, advantages, returns);
    }
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// explained-variance moments {sum y, sum y^2, sum d, sum d^2, n} of y = returns, d = y - values
// (agent :373-377), fp64, one workgroup in a fixed summation order (deterministic); out may be
// host-mapped memory (stored through its device address)
#define VM_THREADS 1024
__global__ __launch_bounds__(VM_THREADS) void value_moments_kernel(const float* __restrict__ val, const float* __restrict__ ret,
                                                                   int64_t n, double* __restrict__ out) {
    __shared__ double sh[4][VM_THREADS / 64];
    double a = 0.0, b = 0.0, c = 0.0, e = 0.0;
    for (int64_t i = threadIdx.x; i < n; i += VM_THREADS) {
        const double y = ret[i], d = y - (double)val[i];
        a += y; b += y * y; c += d; e += d * d;
    }
    a = wave_sumd(a); b = wave_sumd(b); c = wave_sumd(c); e = wave_sumd(e);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) { sh[0][w] = a; sh[1][w] = b; sh[2][w] = c; sh[3][w] = e; }
    __syncthreads();
    if (threadIdx.x < 4) {
        double t = 0.0;
        for (int k = 0; k < VM_THREADS / 64; ++k) t += sh[threadIdx.x][k];
        out[threadIdx.x] = t;
    } else if (threadIdx.x == 4) {
        out[4] = (double)n;
    }
}

extern "C" int dppo_value_moments(const float* values, const float* returns, int64_t n, double* moments, void* stream) {
    DPPO_CHECK(n >= 0 && values && returns && moments, "dppo_value_moments: bad args");
    double* out = moments;
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, moments, 0) == hipSuccess && dp) out = (double*)dp;
    else (void)hipGetLastError();
    hipLaunchKernelGGL(value_moments_kernel, dim3(1), dim3(VM_THREADS), 0, (hipStream_t)stream, values, returns, n, out);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_reward_scale_moments(const double* reward, const uint8_t* first, double* ret_state, double* workspace,
                                         double* moments, int S, int E, double gamma, void* stream) {
    DPPO_CHECK(S > 0 && E > 0, "dppo_reward_scale_moments: empty");
    DPPO_CHECK(reward && first && ret_state && workspace && moments, "dppo_reward_scale_moments: null pointer");
    hipStream_t s = (hipStream_t)stream;
    double* rets_ws = workspace;
    double* env_mom = rets_ws + (size_t)S * E;
    { DppoKtScope kt(KT_RETS, (hipStream_t)stream);
        hipLaunchKernelGGL(rets_kernel, dim3(dppo_cdiv(E, SCAN_WAVES)), dim3(64 * SCAN_WAVES), 0, s,
                           reward, first, ret_state, rets_ws, env_mom, S, E, gamma);
    }
    DPPO_HIP(hipGetLastError());
    { DppoKtScope kt(KT_MOMENTS, (hipStream_t)stream);
        hipLaunchKernelGGL(moments_kernel, dim3(1), dim3(64), 0, s, env_mom, E, moments, (double*)nullptr);
    }
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_reward_scale_apply(double* reward, const double* rms_state, int S, int E, double cliprew,
                                       double epsilon, void* stream) {
    DPPO_CHECK(reward && rms_state, "dppo_reward_scale_apply: null pointer");
    const int64_t n = (int64_t)S * E;
    if (n == 0) return DPPO_OK;
    { DppoKtScope kt(KT_SCALE_APPLY, (hipStream_t)stream);
        hipLaunchKernelGGL(scale_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                           reward, rms_state, n, cliprew, epsilon);
    }
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" size_t dppo_reward_scale_workspace_doubles(int S, int E) {
    // the shared scan (rets [S,E] + per-env moments + 3) and, for per_env, the column moments [S][2]
    return (size_t)S * E + (size_t)3 * E + 3 + (size_t)2 * S;
}

// ---------------------------------------------------------------------------------------------
// per_env = True (util/reward_scaling.py:51-66): the RunningMeanStd has shape (num_envs,) and is
// updated with ret_rms.update(rets) on rets [E, S] (env-major), i.e. with np.mean / np.var over
// axis 0 — the ENVS — so each time column t contributes one (mean_t, var_t) pair with batch count E,
// and the state broadcasts against the S columns by NumPy's rules (shape (E,) needs S == E, or one
// side of length 1). transform() then divides reward [E, S] by sqrt(var + eps) along the last axis.
// The sums run over e in order 0..E-1, as NumPy's add.reduce does over a non-contiguous axis.
// rms layout: fp64 [1 + 2 L] = {count, mean[L], var[L]}.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void col_moments_kernel(const double* __restrict__ rets, int S, int E,
                                                          double* __restrict__ colm) {
    for (int t = blockIdx.x * 256 + threadIdx.x; t < S; t += gridDim.x * 256) {
        double s = 0.0;
        for (int e = 0; e < E; ++e) s += rets[(size_t)t * E + e];
        const double mean = s / (double)E;
        double q = 0.0;
        for (int e = 0; e < E; ++e) {
            const double d = rets[(size_t)t * E + e] - mean;
            q += d * d;
        }
        colm[2 * t] = mean;
        colm[2 * t + 1] = q / (double)E;
    }
}

// RunningMeanStd.update_from_moments (reward_scaling.py:29-39) per output column j < Lo with
// NumPy broadcasting: batch column j (S == 1 -> 0), state entry j (Li == 1 -> 0)
__global__ __launch_bounds__(256) void rms_cols_update_kernel(const double* __restrict__ colm, int S, int E,
                                                              const double* __restrict__ rin, int Li,
                                                              double* __restrict__ rout, int Lo) {
    const double count = rin[0], bc = (double)E;
    const double tot = count + bc;
    for (int j = blockIdx.x * 256 + threadIdx.x; j < Lo; j += gridDim.x * 256) {
        const int t = S == 1 ? 0 : j, l = Li == 1 ? 0 : j;
        const double bm = colm[2 * t], bv = colm[2 * t + 1];
        const double mean = rin[1 + l], var = rin[1 + Li + l];
        const double delta = bm - mean;
        const double m_a = var * count;
        const double m_b = bv * bc;
        const double M2 = m_a + m_b + delta * delta * count * bc / tot;
        rout[1 + j] = mean + delta * bc / tot;
        rout[1 + Lo + j] = M2 / (tot - 1.0);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) rout[0] = tot;
}

// out [C, E] time-major, C = S (Lo == S or Lo == 1) or Lo (S == 1): out[c][e] = clip(reward[s][e] /
// sqrt(var[v] + eps)), s = (S == 1 ? 0 : c), v = (Lo == 1 ? 0 : c)
__global__ __launch_bounds__(256) void scale_cols_kernel(const double* __restrict__ rew, const double* __restrict__ rms,
                                                         int S, int E, int Lo, int C, double cliprew, double eps,
                                                         double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)C * E) return;
    const int c = (int)(i / E), e = (int)(i - (int64_t)c * E);
    const int s = S == 1 ? 0 : c, v = Lo == 1 ? 0 : c;
    double r = rew[(size_t)s * E + e] / sqrt(rms[1 + Lo + v] + eps);
    r = r < -cliprew ? -cliprew : (r > cliprew ? cliprew : r);
    out[i] = r;
}

static int bcast_len(int S, int L) { return S == L ? L : (S == 1 ? L : (L == 1 ? S : -1)); }

extern "C" int dppo_reward_scale_per_env_moments(const double* reward, const uint8_t* first, double* ret_state,
                                                 double* workspace, double* col_moments, int S, int E, double gamma,
                                                 void* stream) {
    DPPO_CHECK(S > 0 && E > 0, "dppo_reward_scale_per_env_moments: empty");
    DPPO_CHECK(reward && first && ret_state && workspace && col_moments, "dppo_reward_scale_per_env_moments: null pointer");
    hipStream_t s = (hipStream_t)stream;
    double* rets = workspace;
    double* env_mom = rets + (size_t)S * E;
    { DppoKtScope kt(KT_RETS, s);
        hipLaunchKernelGGL(rets_kernel, dim3(dppo_cdiv(E, SCAN_WAVES)), dim3(64 * SCAN_WAVES), 0, s,
                           reward, first, ret_state, rets, env_mom, S, E, gamma);
    }
    DPPO_HIP(hipGetLastError());
    { DppoKtScope kt(KT_MOMENTS, s);
        hipLaunchKernelGGL(col_moments_kernel, dim3(dppo_cdiv(S, 256)), dim3(256), 0, s, rets, S, E, col_moments);
    }
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_reward_scale_per_env_apply(const double* reward, const double* rms_state, int S, int E, int L,
                                               double cliprew, double epsilon, double* out, void* stream) {
    DPPO_CHECK(S > 0 && E > 0 && L > 0, "dppo_reward_scale_per_env_apply: empty");
    DPPO_CHECK(reward && rms_state && out, "dppo_reward_scale_per_env_apply: null pointer");
    const int C = bcast_len(S, L);
    DPPO_CHECK(C > 0, "operands could not be broadcast together with shapes (%d,) (%d,)", S, L);
    DPPO_CHECK(out != reward || C == S, "dppo_reward_scale_per_env_apply: S == 1 < L needs a separate [L, E] out");
    hipStream_t s = (hipStream_t)stream;
    { DppoKtScope kt(KT_SCALE_APPLY, s);
        hipLaunchKernelGGL(scale_cols_kernel, dim3(dppo_cdiv(C * E, 256)), dim3(256), 0, s, reward, rms_state, S, E, L,
                           C, cliprew, epsilon, out);
    }
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

extern "C" int dppo_reward_scale_per_env(const double* reward, const uint8_t* first, double* ret_state,
                                         const double* rms_in, int L_in, double* rms_out, double* workspace, int S,
                                         int E, double gamma, double cliprew, double epsilon, double* out,
                                         void* stream) {
    DPPO_CHECK(S > 0 && E > 0 && L_in > 0, "dppo_reward_scale_per_env: empty");
    DPPO_CHECK(rms_in && rms_out && rms_in != rms_out, "dppo_reward_scale_per_env: rms_in and rms_out must differ");
    const int Lo = bcast_len(S, L_in);
    DPPO_CHECK(Lo > 0, "operands could not be broadcast together with shapes (%d,) (%d,)", S, L_in);
    double* colm = workspace + (size_t)S * E + (size_t)3 * E + 3;
    int rc = dppo_reward_scale_per_env_moments(reward, first, ret_state, workspace, colm, S, E, gamma, stream);
    if (rc) return rc;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(rms_cols_update_kernel, dim3(dppo_cdiv(Lo, 256)), dim3(256), 0, s, colm, S, E, rms_in, L_in,
                       rms_out, Lo);
    DPPO_HIP(hipGetLastError());
    return dppo_reward_scale_per_env_apply(reward, rms_out, S, E, Lo, cliprew, epsilon, out, stream);
}

extern "C" int dppo_reward_scale(double* reward, const uint8_t* first, double* ret_state, double* rms_state,
                                 double* workspace, int S, int E, double gamma, double cliprew, double epsilon,
                                 void* stream) {
    DPPO_CHECK(S > 0 && E > 0, "dppo_reward_scale: empty");
    DPPO_CHECK(reward && first && ret_state && rms_state && workspace, "dppo_reward_scale: null pointer");
    hipStream_t s = (hipStream_t)stream;
    double* rets = workspace;
    double* env_mom = rets + (size_t)S * E;
    double* moments = env_mom + (size_t)3 * E;
    { DppoKtScope kt(KT_RETS, (hipStream_t)stream);
        hipLaunchKernelGGL(rets_kernel, dim3(dppo_cdiv(E, SCAN_WAVES)), dim3(64 * SCAN_WAVES), 0, s,
                           reward, first, ret_state, rets, env_mom, S, E, gamma);
    }
    DPPO_HIP(hipGetLastError());
    { DppoKtScope kt(KT_MOMENTS, (hipStream_t)stream);
        hipLaunchKernelGGL(moments_kernel, dim3(1), dim3(64), 0, s, env_mom, E, moments, rms_state);
    }
    DPPO_HIP(hipGetLastError());
    { DppoKtScope kt(KT_SCALE_APPLY, (hipStream_t)stream);
        hipLaunchKernelGGL(scale_apply_kernel, dim3(dppo_cdiv(S * E, 256)), dim3(256), 0, s, reward, rms_state,
                           (int64_t)S * E, cliprew, epsilon);
    }
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}

// ---------------------------------------------------------------------------------------------
// a16 episode accounting (train_ppo_diffusion_agent.py:144-167): the episodes that start AND end
// inside the rollout — consecutive episode starts s < en of one env with en - s > 1 — and per env
// {count, sum of returns (sum of rew[s:en]), sum of best rewards (max of rew[s:en] / act_steps),
// count with best >= threshold}. One lane per env walks t = 0..S in order (the reference's env-major
// visit; per-episode sums in time order), on the RAW rewards (before the reward scaler).
// The caller sums the E rows in env order. (ABI 14: the host loop took ~0.4 ms at 64 envs and
// ~13 ms at 512 inside the update loop, where the host is at most one minibatch ahead of the GPU.)
// ---------------------------------------------------------------------------------------------
// A workgroup owns 64 envs (one walking lane each, wave 0) and streams the [t][env] slab through LDS in
// chunks of EP_CH steps: waves 1-3 load a chunk with coalesced rows (rewards 512 B, flags 64 B per step)
// while wave 0 walks the previous one, so the walk never waits on a global load (one thread per
// env reading its own column paid a load latency per step or per few steps: 208 / 155 us at S = 500,
// against 53.5 us here; tools/r06_ep.sh).
constexpr int EP_ENVS = 64, EP_CH = 32;
__global__ __launch_bounds__(256) void episode_sums_kernel(const double* __restrict__ rew, const uint8_t* __restrict__ first,
                                                           int S, int E, double act_steps, double thr,
                                                           double* __restrict__ out) {
    __shared__ double srew[2][EP_CH][EP_ENVS];
    __shared__ uint8_t sfl[2][EP_CH][EP_ENVS];
    const int tid = (int)threadIdx.x, e0 = (int)blockIdx.x * EP_ENVS, e = e0 + tid;
    const int nch = (S + 1 + EP_CH - 1) / EP_CH;   // chunks over t = 0..S (flags have S + 1 rows)
    auto load = [&](int c, int buf) {   // waves 1-3 (wave 0 walks, never waiting on a load of its own)
        constexpr int LT = 256 - EP_ENVS, NL = (EP_CH * EP_ENVS + LT - 1) / LT;
        double rv[NL];
        uint8_t fv[NL];
#pragma unroll
        for (int k = 0; k < NL; ++k) {   // every load of the chunk issued before the first LDS store
            const int i = tid - EP_ENVS + LT * k, tt = i / EP_ENVS, ee = i % EP_ENVS, t = c * EP_CH + tt, eg = e0 + ee;
            const bool ok = tid >= EP_ENVS && i < EP_CH * EP_ENVS && eg < E;
            rv[k] = ok && t < S ? rew[(size_t)t * E + eg] : 0.0;
            fv[k] = ok && t <= S ? first[(size_t)t * E + eg] : (uint8_t)0;
        }
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int i = tid - EP_ENVS + LT * k;
            if (tid >= EP_ENVS && i < EP_CH * EP_ENVS) {
                srew[buf][i / EP_ENVS][i % EP_ENVS] = rv[k];
                sfl[buf][i / EP_ENVS][i % EP_ENVS] = fv[k];
            }
        }
    };
    int start = -1;
    double run = 0.0, mx = 0.0, n = 0.0, tot = 0.0, best = 0.0, succ = 0.0;
    load(0, 0);
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
        if (c + 1 < nch) load(c + 1, (c + 1) & 1);   // the next chunk in flight during this walk
        if (tid < EP_ENVS) {
            const int buf = c & 1;
#pragma unroll 8
            for (int tt = 0; tt < EP_CH; ++tt) {
                const int t = c * EP_CH + tt;
                if (t <= S && sfl[buf][tt][tid]) {
                    if (start >= 0 && t - start > 1) {
                        const double b = mx / act_steps;
                        n += 1.0;
                        tot += run;
                        best += b;
                        succ += b >= thr ? 1.0 : 0.0;
                    }
                    start = t;
                    run = 0.0;
                    mx = -__builtin_huge_val();
                }
                if (t < S) {
                    const double r = srew[buf][tt][tid];
                    run += r;
                    mx = fmax(mx, r);
                }
            }
        }
        __syncthreads();   // this chunk's buffer is rewritten two chunks on
    }
    if (tid < EP_ENVS && e < E) {
        out[4 * (size_t)e + 0] = n;
        out[4 * (size_t)e + 1] = tot;
        out[4 * (size_t)e + 2] = best;
        out[4 * (size_t)e + 3] = succ;
    }
}

extern "C" int dppo_episode_sums(const double* reward, const uint8_t* first, int S, int E, int act_steps,
                                 double success_threshold, double* out, void* stream) {
    DPPO_CHECK(S >= 0 && E >= 0 && act_steps > 0, "dppo_episode_sums: bad sizes");
    if (E == 0) return DPPO_OK;
    DPPO_CHECK(reward && first && out, "dppo_episode_sums: null pointer");
    hipLaunchKernelGGL(episode_sums_kernel, dim3(dppo_cdiv(E, EP_ENVS)), dim3(256), 0, (hipStream_t)stream, reward, first,
                       S, E, (double)act_steps, success_threshold, out);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}
