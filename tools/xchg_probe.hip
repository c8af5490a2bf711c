// xchg_probe.hip — measures the per-step cost of the split sampler's in-launch partial-sum
// exchange: G groups of P workgroups (one per CU), each step every workgroup publishes 16x12 fp32
// partials as 8-byte {tag, value} granules (sc1 stores), one wave sweeps the P members' granules
// (sc1 loads) until every tag matches, sums them in member order and hands the result to the
// other waves through LDS. Compared against the same loop without the exchange.
//   hipcc --offload-arch=gfx950 -O3 -o tools/xchg_probe tools/xchg_probe.hip && tools/xchg_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NV = 192;   // 16 rows x 12 action coordinates

template <int P, bool XCHG, bool SAMEXCD>
__global__ __launch_bounds__(512) void probe(uint64_t* buf, float* out, uint32_t seq, int steps, int G, int work,
                                             uint32_t* fail) {
    extern __shared__ float lds[];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int g, c;
    if (SAMEXCD) { g = (b / (8 * P)) * 8 + b % 8; c = (b / 8) % P; }
    else { g = b / P; c = b % P; }
    if (g >= G) return;
    float x = (float)(c + 1);
    for (int i = 0; i < steps; ++i) {
        // stand-in for the step's GEMMs
        for (int w = 0; w < work; ++w) __builtin_amdgcn_s_sleep(127);
        const uint32_t tag = seq * 32 + i + 1;
        uint64_t* slot = buf + ((size_t)(i & 1) * G * P + (size_t)g * P) * NV;
        if (XCHG) {
            if (wave == 0) {
                for (int v = lane; v < NV; v += 64) {
                    const float val = x + v;
                    const uint64_t gr = ((uint64_t)tag << 32) | __float_as_uint(val);
                    __hip_atomic_store(slot + (size_t)c * NV + v, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                float s[NV / 64];
                for (int k = 0; k < NV / 64; ++k) s[k] = 0.f;
                uint32_t spins = 0;
                for (;;) {
                    bool ok = true;
                    uint64_t gv[P][NV / 64];
#pragma unroll
                    for (int m = 0; m < P; ++m)
#pragma unroll
                        for (int k = 0; k < NV / 64; ++k) {
                            gv[m][k] = __hip_atomic_load(slot + (size_t)m * NV + lane + 64 * k, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                            ok &= (uint32_t)(gv[m][k] >> 32) == tag;
                        }
                    if (__all(ok)) {
#pragma unroll
                        for (int m = 0; m < P; ++m)
#pragma unroll
                            for (int k = 0; k < NV / 64; ++k) s[k] += __uint_as_float((uint32_t)gv[m][k]);
                        break;
                    }
                    if (++spins > (1u << 22)) { if (lane == 0) atomicAdd(fail, 1u); break; }
                }
                for (int k = 0; k < NV / 64; ++k) lds[lane + 64 * k] = s[k];
            }
            __syncthreads();
            x = lds[(tid % NV)] * 1e-3f;
            __syncthreads();
        } else {
            if (wave == 0) for (int k = 0; k < NV / 64; ++k) lds[lane + 64 * k] = x + k;
            __syncthreads();
            x = lds[(tid % NV)] * 1e-3f;
            __syncthreads();
        }
    }
    if (c == 0 && tid < NV) out[g * NV + tid] = x;
}

template <int P, bool XCHG, bool SAMEXCD>
static int run(const char* name, int G, int work, uint64_t* buf, float* out, uint32_t* fail, uint32_t& seq) {
    const int steps = 20, reps = 50;
    int blocks = G * P;
    if (SAMEXCD) blocks = ((G + 7) / 8) * 8 * P;
    auto k = probe<P, XCHG, SAMEXCD>;
    CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 100 * 1024, 0, buf, out, ++seq, steps, G, work, fail);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 100 * 1024, 0, buf, out, ++seq, steps, G, work, fail);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t f;
    CHECK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
    printf("%-28s P=%d G=%3d work=%d: %7.2f us/launch, %6.3f us/step  fails=%u\n", name, P, G, work,
           1000.f * ms / reps, 1000.f * ms / reps / steps, f);
    return 0;
}

int main() {
    uint64_t* buf; float* out; uint32_t* fail;
    CHECK(hipMalloc(&buf, 2 * 64 * 16 * NV * 8));
    CHECK(hipMemset(buf, 0, 2 * 64 * 16 * NV * 8));
    CHECK(hipMalloc(&out, 64 * NV * 4));
    CHECK(hipMalloc(&fail, 4));
    CHECK(hipMemset(fail, 0, 4));
    uint32_t seq = 0;
    for (int work : {0, 4}) {
        run<8, false, false>("no exchange", 4, work, buf, out, fail, seq);
        run<8, true, false>("exchange, spread", 4, work, buf, out, fail, seq);
        run<8, true, false>("exchange, spread", 8, work, buf, out, fail, seq);
        run<8, true, true>("exchange, same XCD", 8, work, buf, out, fail, seq);
        run<4, true, false>("exchange, spread", 4, work, buf, out, fail, seq);
        run<4, true, true>("exchange, same XCD", 8, work, buf, out, fail, seq);
        run<16, true, false>("exchange, spread", 4, work, buf, out, fail, seq);
        run<8, true, false>("exchange, spread", 32, work, buf, out, fail, seq);
    }
    return 0;
}
