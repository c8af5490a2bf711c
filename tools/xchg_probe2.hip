// xchg_probe2.hip — the split sampler's partial-sum exchange with two store flavours:
//   sc1 : write-through agent-scope granule stores (drop the line from L2; the poller re-reads it
//         from the memory side) — placement-independent, the r01 kernel's form
//   sc0 : workgroup-scope granule stores (the line stays in the producer XCD's L2); the poller's
//         sc1 loads bypass its own L1 and hit that same L2 — valid ONLY when every member of the
//         group runs on one XCD, which each member checks at run time from HW_REG_XCC_ID
// Groups are formed from blockIdx (b % 8 shared inside a group: one XCD under round-robin
// placement) and, for the "cross" rows, deliberately spread over XCDs (expect sc0 to time out there).
//   hipcc --offload-arch=gfx950 -O3 -o tools/xchg_probe2 tools/xchg_probe2.hip && tools/xchg_probe2
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NV = 192;   // 16 rows x 12 action coordinates

__device__ inline int xcc_id() {
    int x;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
    return x;
}

template <int P, bool SC0, bool SAMEXCD>
__global__ __launch_bounds__(512) void probe(uint64_t* buf, float* out, uint32_t seq, int steps, int G, int work,
                                             uint32_t* fail, int* xcc_out) {
    extern __shared__ float lds[];
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int g, c;
    if (SAMEXCD) { g = (b / (8 * P)) * 8 + b % 8; c = (b / 8) % P; }
    else { g = b / P; c = b % P; }
    if (g >= G) return;
    if (tid == 0) xcc_out[g * P + c] = xcc_id();
    float x = (float)(c + 1);
    for (int i = 0; i < steps; ++i) {
        for (int w = 0; w < work; ++w) __builtin_amdgcn_s_sleep(127);
        const uint32_t tag = seq * 64 + i + 1;
        uint64_t* slot = buf + ((size_t)(i & 1) * G * P + (size_t)g * P) * NV;
        // 8 waves publish NV/8 granules each, then sweep NV/8 coordinates from all P members
        const int NVW = NV / 8;
        const int vw = wave * NVW;
        if (lane < NVW) {
            const float val = x + (vw + lane) + c;
            const uint64_t gr = ((uint64_t)tag << 32) | __float_as_uint(val);
            if (SC0) __hip_atomic_store(slot + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            else __hip_atomic_store(slot + (size_t)c * NV + vw + lane, gr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // lane = slot * P + member over (64 / P) slots per pass
        constexpr int SL = 64 / P, KW = (NVW + SL - 1) / SL;
        const int m = lane % P, sl = lane / P;
        float s = 0.f;
        uint32_t spins = 0;
        uint64_t gv[KW];
        for (;;) {
            bool ok = true;
#pragma unroll
            for (int k = 0; k < KW; ++k) {
                const int v = sl + SL * k;
                gv[k] = v < NVW ? __hip_atomic_load(slot + (size_t)m * NV + vw + v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                : ((uint64_t)tag << 32);
                ok &= (uint32_t)(gv[k] >> 32) == tag;
            }
            if (__all(ok)) break;
            if (++spins > (1u << 14)) { if (lane == 0) atomicAdd(fail, 1u); break; }
        }
#pragma unroll
        for (int k = 0; k < KW; ++k) s += __uint_as_float((uint32_t)gv[k]);
        if (lane < NVW) lds[vw + lane] = s;
        __syncthreads();
        x = lds[(tid % NV)] * 1e-3f;
        __syncthreads();
    }
    if (c == 0 && tid < NV) out[g * NV + tid] = x;
}

template <int P, bool SC0, bool SAMEXCD>
static int run(const char* name, int G, int work, uint64_t* buf, float* out, uint32_t* fail, int* xcc, uint32_t& seq,
               int reps = 50) {
    const int steps = 20;
    int blocks = G * P;
    if (SAMEXCD) blocks = ((G + 7) / 8) * 8 * P;
    auto k = probe<P, SC0, SAMEXCD>;
    CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 100 * 1024));
    CHECK(hipMemset(fail, 0, 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    for (int r = 0; r < (reps > 3 ? 3 : 0); ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 100 * 1024, 0, buf, out, ++seq, steps, G, work, fail, xcc);
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(512), 100 * 1024, 0, buf, out, ++seq, steps, G, work, fail, xcc);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    uint32_t f;
    CHECK(hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost));
    int hx[64 * 16];
    CHECK(hipMemcpy(hx, xcc, sizeof(int) * G * P, hipMemcpyDeviceToHost));
    int same = 0;
    for (int g = 0; g < G; ++g) {
        bool s = true;
        for (int c = 1; c < P; ++c) s &= hx[g * P + c] == hx[g * P];
        same += s;
    }
    printf("%-34s P=%2d G=%2d work=%d: %7.2f us/launch %6.3f us/step  groups one-XCD %d/%d  timeouts=%u\n", name, P,
           G, work, 1000.f * ms / reps, 1000.f * ms / reps / steps, same, G, f);
    return 0;
}

int main() {
    uint64_t* buf; float* out; uint32_t* fail; int* xcc;
    CHECK(hipMalloc(&buf, 2 * 64 * 16 * NV * 8));
    CHECK(hipMemset(buf, 0, 2 * 64 * 16 * NV * 8));
    CHECK(hipMalloc(&out, 64 * NV * 4));
    CHECK(hipMalloc(&fail, 4));
    CHECK(hipMalloc(&xcc, 64 * 16 * 4));
    uint32_t seq = 0;
    for (int work : {0}) {
        run<2, true, true>("sc0 stores, one XCD", 4, work, buf, out, fail, xcc, seq);
        run<4, true, true>("sc0 stores, one XCD", 4, work, buf, out, fail, xcc, seq);
        run<4, true, true>("sc0 stores, one XCD", 32, work, buf, out, fail, xcc, seq);
        run<8, false, true>("sc1 stores, one XCD", 4, work, buf, out, fail, xcc, seq);
        run<8, true, true>("sc0 stores, one XCD", 4, work, buf, out, fail, xcc, seq);
        run<16, false, true>("sc1 stores, one XCD", 4, work, buf, out, fail, xcc, seq);
        run<16, true, true>("sc0 stores, one XCD", 4, work, buf, out, fail, xcc, seq);
        run<8, false, true>("sc1 stores, one XCD", 32, work, buf, out, fail, xcc, seq);
        run<8, true, true>("sc0 stores, one XCD", 32, work, buf, out, fail, xcc, seq);
    }
    // spread groups: sc1 works, sc0 is expected to stall until the bounded spin gives up
    run<8, false, false>("sc1 stores, spread over XCDs", 4, 0, buf, out, fail, xcc, seq);
    run<8, true, false>("sc0 stores, spread (expect timeouts)", 1, 0, buf, out, fail, xcc, seq, 1);
    return 0;
}
