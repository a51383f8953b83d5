// Latency microbenchmarks that decide the late-phase design (per-merge kernels vs a persistent loop):
//  - back-to-back launches of an empty kernel at several grid sizes (dispatch + drain per launch)
//  - a dependent pointer chase (one lane) through an array that lives in L2 / Infinity Cache / HBM
//  - a grid barrier (atomic arrive + spin) inside one persistent launch, per barrier
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/launch_lat tools/launch_lat.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

__global__ void empty_k(int *p) { if (p && threadIdx.x == 1023) p[0] = 1; }

// kernels that differ only in what the dispatcher must set up: private (scratch) memory, a large LDS
// allocation; launched in alternating pairs to see which one a kernel boundary charges for
// private memory allocated (the dynamically indexed array) but never touched: idx >= 0 always
template <int N>
__global__ void scratch_k(int *p, int idx) {
    if (idx < 0) {
        int a[N];
        for (int k = 0; k < N; k++) a[k] = k * (int)threadIdx.x;
        p[0] = a[(-idx + threadIdx.x) % N];
    }
}
__global__ void lds_k(int *p) {
    __shared__ uint32_t l[9728];  // 38 KB, like the scan kernel
    l[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p && l[(threadIdx.x + 1) & 255] == 999999u) p[0] = 1;
}

__global__ void stride_init_k(uint32_t *next, uint64_t n, uint64_t stride) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        next[i] = (uint32_t)((i + stride) % n);
}
__global__ void chase_k(const uint32_t *next, int steps, uint32_t *out) {
    uint32_t i = 0;
    for (int s = 0; s < steps; s++) i = __builtin_nontemporal_load(&next[i]);
    out[0] = i;
}

// sense-reversing grid barrier; gives up after ~50 ms of spinning (sets *err) so every wave ends
__device__ bool grid_sync(unsigned *count, unsigned *gen, unsigned nblocks, unsigned *err) {
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned g = __hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __atomic_thread_fence(__ATOMIC_RELEASE);
        if (atomicAdd(count, 1u) == nblocks - 1) {
            __hip_atomic_store(count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(gen, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            const long long t0 = wall_clock64();
            while (__hip_atomic_load(gen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == g) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t0 > 5000000) { atomicOr(err, 1u); break; }  // 100 MHz clock: 50 ms
            }
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    }
    __syncthreads();
    return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

// select_next's end pattern: every block writes `words` u32 per thread, then release fence (agent) +
// ticket; the last block acquires and reads one word per block
// dependent chain of returning device-scope atomics (one lane): each add's address depends on the last result
__global__ void atomic_chain_k(uint32_t *a, int steps, uint32_t *out) {
    uint32_t i = 0;
    for (int s = 0; s < steps; s++) i = (atomicAdd(&a[(i & 1023) * 16], 1u) + s) & 1023;
    out[0] = i;
}
// the same with LDS atomics
__global__ void lds_chain_k(int steps, uint32_t *out) {
    __shared__ uint32_t l[1024];
    for (int k = threadIdx.x; k < 1024; k += blockDim.x) l[k] = 0;
    __syncthreads();
    uint32_t i = 0;
    if (threadIdx.x == 0)
        for (int s = 0; s < steps; s++) i = (atomicAdd(&l[i & 1023], 1u) + s) & 1023;
    if (threadIdx.x == 0) out[0] = i;
}

template <bool FENCE>
__global__ void ticket_k(uint32_t *data, int words, unsigned *ticket, uint32_t *out) {
    __shared__ unsigned s_last;
    for (int k = 0; k < words; k++) data[((size_t)blockIdx.x * words + k) * blockDim.x + threadIdx.x] = k + threadIdx.x;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool last = t == gridDim.x - 1;
        if (last && FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_last = last;
    }
    __syncthreads();
    if (!s_last) return;
    uint32_t acc = 0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += blockDim.x) acc += data[(size_t)b * words * blockDim.x];
    if (acc == 12345) out[0] = acc;
    if (threadIdx.x == 0) *ticket = 0;
}

__global__ void barrier_k(unsigned *count, unsigned *gen, int iters, unsigned *err) {
    for (int i = 0; i < iters; i++)
        if (!grid_sync(count, gen, gridDim.x, err)) return;
}

// GPU-side kernel boundary: kernel A spins `spin` ticks, may dirty `dirty` words per block with plain
// stores, and its last block to finish stamps the end (atomicMax); kernel B's first block stamps its start
// (atomicMin). A is long enough for the host to run ahead, so B is queued when A ends.
__global__ void bnd_a(unsigned long long *t, uint32_t *junk, int dirty, long long spin) {
    const long long t0 = wall_clock64();
    while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
    for (int k = 0; k < dirty; k++) junk[((size_t)blockIdx.x * dirty + k) * blockDim.x + threadIdx.x] = k;
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&t[0], (unsigned long long)wall_clock64());
}
__global__ void bnd_b(unsigned long long *t) {
    if (threadIdx.x == 0) atomicMin(&t[1], (unsigned long long)wall_clock64());
}
// the same hand-off inside one launch: blocks [0, na) spin and arrive on a counter (after their stores
// drain), blocks [na, ...) wait for all arrivals (sc1 polls) and stamp
__global__ void bnd_fused(unsigned long long *t, uint32_t *junk, int dirty, long long spin, uint32_t na, uint32_t *ctr) {
    if (blockIdx.x < na) {
        const long long t0 = wall_clock64();
        while (wall_clock64() - t0 < spin) __builtin_amdgcn_s_sleep(1);
        for (int k = 0; k < dirty; k++)
            __hip_atomic_store(&junk[((size_t)blockIdx.x * dirty + k) * blockDim.x + threadIdx.x], (uint32_t)k, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            atomicMax(&t[0], (unsigned long long)wall_clock64());
            __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    if (threadIdx.x == 0) {
        const long long t0 = wall_clock64();
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < na && wall_clock64() - t0 < 5000000)
            __builtin_amdgcn_s_sleep(1);
        atomicMin(&t[1], (unsigned long long)wall_clock64());
    }
}

int main() {
    hipStream_t s;
    CK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms;
    const int R = 2000;
    for (int grid : {1, 64, 256, 1024, 2048, 8192}) {
        for (int w = 0; w < 2; w++) {
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < R; r++) empty_k<<<grid, 256, 0, s>>>(nullptr);
            CK(hipEventRecord(e1, s));
            CK(hipEventSynchronize(e1));
        }
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"test\": \"empty_launch\", \"grid\": %d, \"us_per_launch\": %.3f}\n", grid, ms * 1e3 / R);
    }
    // kernel pairs: which setup does a boundary charge for
    for (int pa = 0; pa < 3; pa++)
        for (int pb = 0; pb < 2; pb++) {
            for (int w = 0; w < 2; w++) {
                CK(hipEventRecord(e0, s));
                for (int r = 0; r < R; r++) {
                    if (pa == 1) scratch_k<64><<<256, 256, 0, s>>>(nullptr, r);
                    else if (pa == 2) scratch_k<256><<<256, 256, 0, s>>>(nullptr, r);
                    else empty_k<<<256, 256, 0, s>>>(nullptr);
                    if (pb) lds_k<<<256, 256, 0, s>>>(nullptr);
                    else empty_k<<<256, 256, 0, s>>>(nullptr);
                }
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
            }
            CK(hipEventElapsedTime(&ms, e0, e1));
            printf("{\"test\": \"pair\", \"first\": \"%s\", \"second\": \"%s\", \"us_per_pair\": %.3f}\n", pa == 1 ? "scratch256B" : pa == 2 ? "scratch1KB" : "empty",
                   pb ? "lds38k" : "empty", ms * 1e3 / R);
        }
    // pointer chase: random cycle over n words
    for (size_t bytes : {(size_t)1 << 20, (size_t)64 << 20, (size_t)512 << 20}) {
        const size_t n = bytes / 4;
        std::vector<uint32_t> h(n);
        std::vector<uint32_t> perm(n);
        for (size_t i = 0; i < n; i++) perm[i] = (uint32_t)i;
        srand(1);
        for (size_t i = n - 1; i > 0; i--) { size_t j = ((size_t)rand() * 65536u + rand()) % (i + 1); std::swap(perm[i], perm[j]); }
        for (size_t i = 0; i < n; i++) h[perm[i]] = perm[(i + 1) % n];
        uint32_t *d, *o;
        CK(hipMalloc(&d, bytes));
        CK(hipMalloc(&o, 4));
        CK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
        const int steps = 20000;
        chase_k<<<1, 1, 0, s>>>(d, steps, o);
        CK(hipEventRecord(e0, s));
        chase_k<<<1, 1, 0, s>>>(d, steps, o);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"test\": \"chase\", \"bytes\": %zu, \"ns_per_load\": %.1f}\n", bytes, ms * 1e6 / steps);
        CK(hipFree(d));
        CK(hipFree(o));
    }
    // pointer chase with a page-sized stride over large buffers: every step touches another 2 MiB page, so
    // the latency includes a GPU TLB miss once the pages outnumber what the TLBs hold
    for (size_t bytes : {(size_t)64 << 20, (size_t)512 << 20, (size_t)2 << 30, (size_t)8 << 30}) {
        const uint64_t n = bytes / 4, stride = ((2u << 20) * 37 + 64) / 4;
        uint32_t *d, *o;
        if (hipMalloc(&d, bytes) != hipSuccess) { printf("{\"test\": \"chase_pages\", \"bytes\": %zu, \"error\": \"alloc\"}\n", bytes); continue; }
        CK(hipMalloc(&o, 4));
        stride_init_k<<<4096, 256, 0, s>>>(d, n, stride);
        const int steps = 20000;
        chase_k<<<1, 1, 0, s>>>(d, steps, o);
        CK(hipEventRecord(e0, s));
        chase_k<<<1, 1, 0, s>>>(d, steps, o);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"test\": \"chase_pages\", \"bytes\": %zu, \"stride_bytes\": %llu, \"ns_per_load\": %.1f}\n", bytes,
               (unsigned long long)stride * 4, ms * 1e6 / steps);
        CK(hipFree(d));
        CK(hipFree(o));
    }
    {
        uint32_t *data, *out;
        unsigned *tk;
        CK(hipMalloc(&data, (size_t)256 << 20));
        CK(hipMalloc(&out, 4));
        CK(hipMalloc(&tk, 4));
        CK(hipMemset(tk, 0, 4));
        for (int fence = 0; fence < 2; fence++)
            for (int grid : {16, 64, 256})
                for (int words : {1, 16, 64}) {
                    const int iters = 500;
                    for (int w = 0; w < 2; w++) {
                        CK(hipEventRecord(e0, s));
                        for (int i = 0; i < iters; i++) {
                            if (fence) ticket_k<true><<<grid, 1024, 0, s>>>(data, words, tk, out);
                            else ticket_k<false><<<grid, 1024, 0, s>>>(data, words, tk, out);
                        }
                        CK(hipEventRecord(e1, s));
                        CK(hipEventSynchronize(e1));
                    }
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    printf("{\"test\": \"ticket\", \"fence\": %d, \"grid\": %d, \"dirty_KB_per_block\": %d, \"us_per_launch\": %.3f}\n",
                           fence, grid, words * 4, ms * 1e3 / iters);
                }
        CK(hipFree(data));
    }
    {
        uint32_t *a, *o;
        CK(hipMalloc(&a, 1024 * 16 * 4));
        CK(hipMalloc(&o, 4));
        CK(hipMemset(a, 0, 1024 * 16 * 4));
        const int steps = 20000;
        atomic_chain_k<<<1, 1, 0, s>>>(a, 100, o);
        CK(hipEventRecord(e0, s));
        atomic_chain_k<<<1, 1, 0, s>>>(a, steps, o);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"test\": \"atomic_chain\", \"ns_per_atomic\": %.1f}\n", ms * 1e6 / steps);
        CK(hipEventRecord(e0, s));
        lds_chain_k<<<1, 64, 0, s>>>(steps, o);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"test\": \"lds_atomic_chain\", \"ns_per_atomic\": %.1f}\n", ms * 1e6 / steps);
        CK(hipFree(a));
    }
    {  // GPU-side boundary between dependent kernels, and the in-launch hand-off
        unsigned long long *t;
        uint32_t *junk, *ctr;
        CK(hipMalloc(&t, 16));
        CK(hipMalloc(&junk, (size_t)64 << 20));
        CK(hipMalloc(&ctr, 4));
        for (int fused = 0; fused < 2; fused++)
            for (int ga : {8, 64, 256})
                for (int gb : {8, 256})
                    for (int dirty : {0, 16}) {
                        double sum = 0;
                        const int reps = 50;
                        for (int r = 0; r < reps; r++) {
                            unsigned long long h[2] = {0, ~0ull};
                            CK(hipMemcpyAsync(t, h, 16, hipMemcpyHostToDevice, s));
                            CK(hipMemsetAsync(ctr, 0, 4, s));
                            if (fused) {
                                bnd_fused<<<ga + gb, 256, 0, s>>>(t, junk, dirty, 2000, ga, ctr);
                            } else {
                                bnd_a<<<ga, 256, 0, s>>>(t, junk, dirty, 2000);
                                bnd_b<<<gb, 256, 0, s>>>(t);
                            }
                            CK(hipMemcpyAsync(h, t, 16, hipMemcpyDeviceToHost, s));
                            CK(hipStreamSynchronize(s));
                            if (r) sum += (double)(h[1] - h[0]) * 0.01;  // 100 MHz ticks -> us
                        }
                        printf("{\"test\": \"boundary\", \"form\": \"%s\", \"grid_a\": %d, \"grid_b\": %d, \"dirty_KB_per_block\": %d, \"us_end_to_start\": %.3f}\n",
                               fused ? "in-launch counter" : "kernel boundary", ga, gb, dirty * 1, sum / (reps - 1));
                    }
        CK(hipFree(t));
        CK(hipFree(junk));
        CK(hipFree(ctr));
    }
    // grid barrier: all blocks resident (grid <= CUs)
    unsigned *cnt, *gen, *err;
    CK(hipMalloc(&cnt, 4)); CK(hipMalloc(&gen, 4)); CK(hipMalloc(&err, 4));
    for (int grid : {8, 32, 64, 128, 256, 512, 1024}) {
        CK(hipMemset(cnt, 0, 4)); CK(hipMemset(gen, 0, 4)); CK(hipMemset(err, 0, 4));
        const int iters = 2000;
        barrier_k<<<grid, 256, 0, s>>>(cnt, gen, 10, err);
        CK(hipEventRecord(e0, s));
        barrier_k<<<grid, 256, 0, s>>>(cnt, gen, iters, err);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        unsigned herr = 0;
        CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
        printf("{\"test\": \"grid_barrier\", \"grid\": %d, \"us_per_barrier\": %.3f, \"err\": %u}\n", grid, ms * 1e3 / iters, herr);
    }
    return 0;
}
