// Read-pattern probe for the dW kernel's operand stream: every CU streams a 256 MB
// feature-major bf16 image set with (A) the current pattern - one 1 KiB wave-instruction = 8 feature
// lines x 128 B, the lines ldm*2 bytes apart - or (B) a row-blocked layout - one wave-instruction =
// 1 KiB contiguous. Reports GB/s of each. hipcc --offload-arch=gfx950 -O3 -o tools/dw_pattern_probe tools/dw_pattern_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// F features x ldm rows of bf16; workgroup g takes features [128 g', ...) and rows [chunk)
template <bool BLOCKED>
__global__ __launch_bounds__(512) void probe(const uint8_t* __restrict__ img, int F, size_t ldm, int nchunks, size_t mchunk,
                                             u32x4* out) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ftiles = F / 64;                       // 64 features per workgroup tile (8 waves x 8 features)
    const int wg = blockIdx.x;
    const int chunk = wg % nchunks, ft = wg / nchunks;
    if (ft >= ftiles) return;
    const int f = ft * 64 + wave * 8 + lane / 8;     // this lane's feature
    const int c = lane % 8;                          // 16-B chunk of the 128-B line
    const size_t m0 = (size_t)chunk * mchunk, m1 = m0 + mchunk < ldm ? m0 + mchunk : ldm;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t m = m0; m < m1; m += 64 * 4) {       // 4 stages of 64 rows in flight per iteration
        u32x4 v[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const size_t r = m + 64 * s;
            size_t off;
            if (BLOCKED) off = ((r / 64) * (size_t)F + f) * 128 + 16 * c;     // [block][f][64 rows]
            else off = ((size_t)f * ldm + r) * 2 + 16 * c;                    // [f][ldm]
            v[s] = r < m1 ? *(const u32x4*)(img + off) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) acc ^= v[s];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = acc;
}

int main() {
    const int F = 2560;                 // 5 x 512 features
    const size_t ldm = 50048;
    const size_t bytes = (size_t)F * ldm * 2;
    uint8_t* img; u32x4* out;
    hipMalloc(&img, bytes + 4096); hipMalloc(&out, 64);
    hipMemset(img, 1, bytes);
    const int nchunks = 16;
    const size_t mchunk = (ldm + nchunks * 64 - 1) / (nchunks * 64) * 64;
    const int grid = (F / 64) * nchunks;
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    for (int pass = 0; pass < 2; ++pass)
        for (int b = 0; b < 2; ++b) {
            for (int w = 0; w < 3; ++w) {
                if (b) probe<true><<<grid, 512>>>(img, F, ldm, nchunks, mchunk, out);
                else probe<false><<<grid, 512>>>(img, F, ldm, nchunks, mchunk, out);
            }
            hipEventRecord(e0);
            const int reps = 20;
            for (int i = 0; i < reps; ++i) {
                if (b) probe<true><<<grid, 512>>>(img, F, ldm, nchunks, mchunk, out);
                else probe<false><<<grid, 512>>>(img, F, ldm, nchunks, mchunk, out);
            }
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1);
            ms /= reps;
            printf("%s: %.1f us, %.2f TB/s\n", b ? "blocked [blk][f][64]" : "feature-major [f][ldm]", ms * 1e3,
                   bytes / (ms * 1e-3) / 1e12);
        }
    return 0;
}
