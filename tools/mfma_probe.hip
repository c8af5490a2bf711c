// Probe of the f32-input MFMA operand maps on gfx950 (diagnostic, not part of the library).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void probe(const float* A, const float* B, float* C, int variant) {
    int l = threadIdx.x;
    f32x4 c = {0, 0, 0, 0};
    // A is 16x4 row-major, B is 4x16 row-major
    float a = A[(l & 15) * 4 + (l >> 4)];
    float b = B[(l >> 4) * 16 + (l & 15)];
    c = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) C[(((l >> 4) << 2) + r) * 16 + (l & 15)] = c[r];
}
int main() {
    float hA[64], hB[64], hC[256], ref[256];
    for (int i = 0; i < 64; ++i) { hA[i] = (float)((i * 7) % 13) - 6; hB[i] = (float)((i * 5) % 11) - 5; }
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { float s = 0; for (int k = 0; k < 4; ++k) s += hA[i * 4 + k] * hB[k * 16 + j]; ref[i * 16 + j] = s; }
    float *A, *B, *C;
    hipMalloc(&A, 256); hipMalloc(&B, 256); hipMalloc(&C, 1024);
    hipMemcpy(A, hA, 256, hipMemcpyHostToDevice); hipMemcpy(B, hB, 256, hipMemcpyHostToDevice);
    probe<<<1, 64>>>(A, B, C, 0);
    hipMemcpy(hC, C, 1024, hipMemcpyDeviceToHost);
    double e = 0; for (int i = 0; i < 256; ++i) e = fmax(e, fabs(hC[i] - ref[i]));
    printf("16x16x4f32 max err %g (C[0]=%g ref %g, C[17]=%g ref %g)\n", e, hC[0], ref[0], hC[17], ref[17]);
    // transposed-C hypothesis
    double et = 0; for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) et = fmax(et, fabs(hC[j * 16 + i] - ref[i * 16 + j]));
    printf("transposed err %g\n", et);
    return 0;
}
