// collective.hip — the data-parallel gradient all-reduce as ONE kernel over
// IPC-mapped peer buffers, the alternative to RCCL's all_reduce for the per-minibatch buckets of the
// split update (agent/finetune/train_ppo_diffusion_agent.py; the reference has no collective: it
// applies gradients on one device, agent :345-356, script/run.py:82).
//
// Every rank owns one region in its HBM (hipExtMallocWithFlags(hipDeviceMallocUncached): fine-grained,
// never held in an L2, so a peer's stores over xGMI and this rank's loads meet in memory; exported with
// hipIpcGetMemHandle, the handles exchanged once over torch.distributed and opened by every peer):
//   [0, 512)        flags F[y] (uint64, 64 B apart): the last barrier value rank y signalled here
//   [2048, 2176)    two ticket counters of this rank's own workgroups (zero between launches)
//   [3072, 3076)    abort word: set by any workgroup of any rank whose barrier wait timed out
//   [4096, ...)     two slots of `capacity` floats (call g uses slot g & 1)
// One launch of ipc_allreduce_kernel on every rank (a two-shot all-reduce):
//   A  copy the local data into the own slot; barrier (value 2g + 1)
//   B  rank r reduces ITS slice r of every rank's slot, in rank order 0..W-1 (plain fp32 adds, so
//      the sum is the same bits on every rank and equals a sequential NumPy float32 sum), and
//      writes the result into that slice of every rank's slot; barrier (value 2g + 2)
//   C  copy the own slot (now fully reduced) back into the local data.
// Every phase moves 16 B per lane (dwordx4 loads and stores, 1 KiB per wave instruction; a ragged
// tail of n % 4 floats by scalar lanes); the grid is sized to the bucket (one float4 per thread
// per pass, at most IPC_MAXB workgroups).
// A barrier: every workgroup waits for its own stores (vmcnt(0)), fences at system scope and takes a
// ticket; the last one stores the barrier value into flag r of every peer's region (system-scope
// release); then every workgroup polls its own region's W flags until each holds at least that value
// (bounded: ~2 s). A workgroup whose wait times out sets the abort word of every rank's region and the
// mapped failure word; every poller also watches its own abort word, so all workgroups of all ranks
// leave together (no sibling waits out its own 2 s, no peer spins on). The host reads the failure
// word before the next call and at the end of every update (util/ipc.py check()). Slots alternate per
// call, so a peer's phase-A copy of call g+1 never overwrites a slot another peer still reads for
// call g (call g+1's first barrier needs every peer done with call g). Traffic per rank per call: n
// floats local in and out, (W-1)/W n remote reads and (W-1)/W n remote writes.
// Written for xGMI peers (one process per GPU); exercised on this pool with 2 and 4 processes that
// share one GPU (same-device IPC). UNMEASURED ON xGMI: RCCL stays the default (train.allreduce).
#include <string.h>
#include "dppo_common.cuh"
#include "dppo_internal.h"

constexpr int IPC_MAXW = 8;
constexpr size_t IPC_HDR = 4096;
constexpr int IPC_MAXB = 64;
static_assert(sizeof(hipIpcMemHandle_t) == 64, "HIP IPC handles are 64 bytes");

struct IpcArgs {
    uint8_t* reg[IPC_MAXW];   // regions as mapped in this process; reg[r] = this rank's own
    float* data;
    int64_t n, cap;
    int W, r;
    uint64_t gen;
    uint32_t* fail;           // mapped host word (device address)
};

__device__ inline uint64_t* ipc_flag(uint8_t* reg, int y) { return reinterpret_cast<uint64_t*>(reg + 64 * y); }
__device__ inline unsigned* ipc_ticket(uint8_t* reg, int k) { return reinterpret_cast<unsigned*>(reg + 2048 + 64 * k); }
__device__ inline unsigned* ipc_abort(uint8_t* reg) { return reinterpret_cast<unsigned*>(reg + 3072); }
__device__ inline float* ipc_slot(uint8_t* reg, int slot, int64_t cap) {
    return reinterpret_cast<float*>(reg + IPC_HDR) + (size_t)slot * cap;
}

// every workgroup of this rank, then every rank: see the file comment. false on a timeout or an abort
__device__ inline bool ipc_barrier(const IpcArgs& a, int k, uint64_t value) {
    __shared__ int ok_s;
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this thread's slot stores have completed
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();   // this workgroup's slot writes (own and peers') before its ticket
        unsigned* t = ipc_ticket(a.reg[a.r], k);
        if (__hip_atomic_fetch_add(t, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
            __hip_atomic_store(t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __threadfence_system();
            for (int x = 0; x < a.W; ++x)
                __hip_atomic_store(ipc_flag(a.reg[x], a.r), value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        ok_s = 1;
    }
    __syncthreads();
    if ((int)threadIdx.x < a.W) {
        const uint64_t t_end = __builtin_amdgcn_s_memrealtime() + 200000000ull;   // 2 s (100 MHz)
        const uint64_t* f = ipc_flag(a.reg[a.r], threadIdx.x);
        const unsigned* ab = ipc_abort(a.reg[a.r]);
        while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < value) {
            if (__hip_atomic_load(ab, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) { ok_s = 0; break; }
            if (__builtin_amdgcn_s_memrealtime() > t_end) {
                ok_s = 0;
                for (int x = 0; x < a.W; ++x)   // every workgroup of every rank leaves now
                    __hip_atomic_store(ipc_abort(a.reg[x]), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(a.fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    __syncthreads();
    __threadfence_system();       // acquire: the peers' slot writes before their flags
    return ok_s != 0;
}

__global__ __launch_bounds__(256) void ipc_allreduce_kernel(IpcArgs a) {
    const int slot = (int)(a.gen & 1);
    const int64_t stride = (int64_t)gridDim.x * 256, t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t n4 = a.n >> 2;                       // whole float4s; the tail n % 4 by scalar lanes
    float* own = ipc_slot(a.reg[a.r], slot, a.cap);
    const bool vec = ((uintptr_t)a.data & 15) == 0;    // the local bucket: 16-B aligned, or scalar copies
    if (vec) {
        for (int64_t i = t0; i < n4; i += stride) reinterpret_cast<float4*>(own)[i] = reinterpret_cast<const float4*>(a.data)[i];
        if (t0 < (a.n & 3)) own[4 * n4 + t0] = a.data[4 * n4 + t0];
    } else {
        for (int64_t i = t0; i < a.n; i += stride) own[i] = a.data[i];
    }
    if (!ipc_barrier(a, 0, 2 * a.gen + 1)) return;
    // slice r of the W slices (whole float4s: `per` is a multiple of 4 elements)
    const int64_t per = ((a.n + a.W - 1) / a.W + 3) & ~(int64_t)3;
    const int64_t lo = per * a.r, hi = lo + per < a.n ? lo + per : a.n;
    const int64_t hi4 = lo + ((hi > lo ? hi - lo : 0) & ~(int64_t)3);
    for (int64_t i = lo / 4 + t0; i < hi4 / 4; i += stride) {
        float4 s = reinterpret_cast<const float4*>(ipc_slot(a.reg[0], slot, a.cap))[i];
        for (int x = 1; x < a.W; ++x) {
            const float4 v = reinterpret_cast<const float4*>(ipc_slot(a.reg[x], slot, a.cap))[i];
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
        }
        for (int x = 0; x < a.W; ++x) reinterpret_cast<float4*>(ipc_slot(a.reg[x], slot, a.cap))[i] = s;
    }
    if (t0 < hi - hi4) {   // the last slice's ragged tail
        const int64_t i = hi4 + t0;
        float s = ipc_slot(a.reg[0], slot, a.cap)[i];
        for (int x = 1; x < a.W; ++x) s += ipc_slot(a.reg[x], slot, a.cap)[i];
        for (int x = 0; x < a.W; ++x) ipc_slot(a.reg[x], slot, a.cap)[i] = s;
    }
    if (!ipc_barrier(a, 1, 2 * a.gen + 2)) return;
    if (vec) {
        for (int64_t i = t0; i < n4; i += stride) reinterpret_cast<float4*>(a.data)[i] = reinterpret_cast<const float4*>(own)[i];
        if (t0 < (a.n & 3)) a.data[4 * n4 + t0] = own[4 * n4 + t0];
    } else {
        for (int64_t i = t0; i < a.n; i += stride) a.data[i] = own[i];
    }
}

extern "C" size_t dppo_ipc_region_bytes(int64_t capacity) {
    return capacity < 0 ? 0 : IPC_HDR + (size_t)2 * (size_t)((capacity + 3) & ~(int64_t)3) * sizeof(float);
}

extern "C" int dppo_ipc_alloc(size_t bytes, void** ptr, void* handle) {
    DPPO_CHECK(ptr && handle && bytes >= IPC_HDR, "dppo_ipc_alloc: bad arguments");
    // uncached (fine-grained): no L2 of the owner's device holds a line a peer writes over the link
    DPPO_HIP(hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached));
    DPPO_HIP(hipMemset(*ptr, 0, bytes));
    hipIpcMemHandle_t h;
    DPPO_HIP(hipIpcGetMemHandle(&h, *ptr));
    memcpy(handle, &h, sizeof(h));
    return DPPO_OK;
}

extern "C" int dppo_ipc_open(const void* handle, void** ptr) {
    DPPO_CHECK(handle && ptr, "dppo_ipc_open: bad arguments");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    DPPO_HIP(hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess));
    return DPPO_OK;
}

extern "C" int dppo_ipc_close(void* ptr) {
    if (ptr) DPPO_HIP(hipIpcCloseMemHandle(ptr));
    return DPPO_OK;
}

extern "C" int dppo_ipc_free(void* ptr) {
    if (ptr) DPPO_HIP(hipFree(ptr));
    return DPPO_OK;
}

extern "C" int dppo_ipc_allreduce(void* const* regions, int world, int rank, int64_t capacity, float* data, int64_t n,
                                  uint64_t generation, uint32_t* fail_host, void* stream) {
    DPPO_CHECK(regions && world >= 1 && world <= IPC_MAXW && rank >= 0 && rank < world,
               "dppo_ipc_allreduce: world must be in [1, %d] and rank < world", IPC_MAXW);
    DPPO_CHECK(n >= 0 && n <= capacity && (n == 0 || data), "dppo_ipc_allreduce: n outside [0, capacity]");
    DPPO_CHECK(generation >= 1 && generation < ((uint64_t)1 << 62), "dppo_ipc_allreduce: generation must be >= 1");
    DPPO_CHECK(fail_host, "dppo_ipc_allreduce: a mapped failure word (dppo_host_alloc) is required");
    if (__hip_atomic_load(fail_host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM))
        return dppo_set_error(DPPO_EHIP, "dppo_ipc_allreduce: an earlier call's barrier timed out (a peer did not "
                                         "arrive); the group's results are not valid");
    IpcArgs a = {};
    for (int x = 0; x < world; ++x) {
        DPPO_CHECK(regions[x], "dppo_ipc_allreduce: region %d is NULL", x);
        a.reg[x] = (uint8_t*)regions[x];
    }
    a.data = data; a.n = n; a.cap = (capacity + 3) & ~(int64_t)3; a.W = world; a.r = rank; a.gen = generation;
    void* dp = nullptr;
    DPPO_HIP(hipHostGetDevicePointer(&dp, fail_host, 0));
    a.fail = (uint32_t*)dp;
    // one float4 per thread per pass, the grid sized to the bucket
    const int64_t want = (n / 4 + 255) / 256;
    const unsigned blocks = (unsigned)(want < 1 ? 1 : (want < IPC_MAXB ? want : IPC_MAXB));
    DppoKtScope kt(KT_ALLREDUCE, (hipStream_t)stream);
    hipLaunchKernelGGL(ipc_allreduce_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, a);
    DPPO_HIP(hipGetLastError());
    return DPPO_OK;
}
