// Micro-benchmark: cost of wave-aggregated queue appends (one global atomic
// per wave per counter) vs block-aggregated (one per block) vs none, in the
// shape of k_step: 2048 blocks x 256 threads, 4 strided chunks each, 6 counters.
#include <hip/hip_runtime.h>
#include <cstdio>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

__global__ __launch_bounds__(256) void k_wave(int* cnt, int* out, int n, int ncnt)
{
    for (int base = (blockIdx.x * 256 + threadIdx.x) & ~63; base < n; base += gridDim.x * 256) {
        const int i = base + (threadIdx.x & 63);
        for (int k = 0; k < ncnt; k++) {
            const bool want = ((i * 2654435761u) >> (k + 3)) & 1;
            const unsigned long long b = __ballot(want);
            int off = 0;
            if ((threadIdx.x & 63) == 0) off = atomicAdd(cnt + k * 32, __popcll(b));
            off = __shfl(off, 0);
            if (want) out[(size_t)k * n + ((off + __popcll(b & ((1ull << (threadIdx.x & 63)) - 1))) % n)] = i;
        }
    }
}

// wave-aggregated, counters sharded by chunk (chunk % S), 128-B apart
template <int S>
__global__ __launch_bounds__(256) void k_shard(int* cnt, int* out, int n, int ncnt)
{
    for (int base = (blockIdx.x * 256 + threadIdx.x) & ~63; base < n; base += gridDim.x * 256) {
        const int i = base + (threadIdx.x & 63);
        const int sh = (base >> 6) % S;
        for (int k = 0; k < ncnt; k++) {
            const bool want = ((i * 2654435761u) >> (k + 3)) & 1;
            const unsigned long long b = __ballot(want);
            int off = 0;
            if ((threadIdx.x & 63) == 0) off = atomicAdd(cnt + (k * S + sh) * 32, __popcll(b));
            off = __shfl(off, 0);
            if (want) out[(size_t)k * n + ((sh * (n / S) + off + __popcll(b & ((1ull << (threadIdx.x & 63)) - 1))) % n)] = i;
        }
    }
}

__global__ __launch_bounds__(256) void k_block(int* cnt, int* out, int n, int ncnt)
{
    __shared__ int s_cnt[8], s_base[8];
    for (int base = blockIdx.x * 256; base < n + 0; base += gridDim.x * 256) {
        const int i = base + threadIdx.x;
        for (int k = 0; k < ncnt; k++) {
            if (threadIdx.x == 0) s_cnt[k] = 0;
            __syncthreads();
            const bool want = ((i * 2654435761u) >> (k + 3)) & 1;
            const unsigned long long b = __ballot(want);
            int woff = 0;
            if ((threadIdx.x & 63) == 0) woff = atomicAdd(&s_cnt[k], __popcll(b));
            woff = __shfl(woff, 0);
            __syncthreads();
            if (threadIdx.x == 0) s_base[k] = atomicAdd(cnt + k * 32, s_cnt[k]);
            __syncthreads();
            if (want) out[(size_t)k * n + ((s_base[k] + woff + __popcll(b & ((1ull << (threadIdx.x & 63)) - 1))) % n)] = i;
        }
    }
}

__global__ __launch_bounds__(256) void k_none(int* cnt, int* out, int n, int ncnt)
{
    for (int base = blockIdx.x * 256; base < n; base += gridDim.x * 256) {
        const int i = base + threadIdx.x;
        for (int k = 0; k < ncnt; k++) {
            const bool want = ((i * 2654435761u) >> (k + 3)) & 1;
            if (want) out[(size_t)k * n + i] = i;
        }
    }
}

int main()
{
    const int n = 1920 * 1080, ncnt = 6;
    int *cnt, *out;
    CHK(hipMalloc(&cnt, 1 << 20));
    CHK(hipMalloc(&out, (size_t)n * ncnt * 4));
    hipEvent_t a, b;
    CHK(hipEventCreate(&a));
    CHK(hipEventCreate(&b));
    for (int grid : {256, 1024, 2048, 8100}) {
        for (int v = 0; v < 6; v++) {
            float best = 1e9;
            for (int rep = 0; rep < 20; rep++) {
                CHK(hipMemset(cnt, 0, 1 << 20));
                CHK(hipEventRecord(a));
                if (v == 0) hipLaunchKernelGGL(k_none, dim3(grid), dim3(256), 0, 0, cnt, out, n, ncnt);
                if (v == 1) hipLaunchKernelGGL(k_wave, dim3(grid), dim3(256), 0, 0, cnt, out, n, ncnt);
                if (v == 2) hipLaunchKernelGGL(k_block, dim3(grid), dim3(256), 0, 0, cnt, out, n, ncnt);
                if (v == 3) hipLaunchKernelGGL(k_shard<8>, dim3(grid), dim3(256), 0, 0, cnt, out, n, ncnt);
                if (v == 4) hipLaunchKernelGGL(k_shard<64>, dim3(grid), dim3(256), 0, 0, cnt, out, n, ncnt);
                if (v == 5) hipLaunchKernelGGL(k_shard<256>, dim3(grid), dim3(256), 0, 0, cnt, out, n, ncnt);
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                float ms;
                CHK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            printf("grid %5d %-6s %8.1f us\n", grid, v == 0 ? "none" : v == 1 ? "wave" : v == 2 ? "block" : v == 3 ? "shard8" : v == 4 ? "shard64" : "shard256", best * 1e3);
        }
    }
    // empty-launch floor
    float best = 1e9;
    for (int rep = 0; rep < 20; rep++) {
        CHK(hipEventRecord(a));
        hipLaunchKernelGGL(k_none, dim3(2048), dim3(256), 0, 0, cnt, out, 0, ncnt);
        CHK(hipEventRecord(b));
        CHK(hipEventSynchronize(b));
        float ms;
        CHK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) best = ms;
    }
    printf("empty launch (2048 blocks) %.1f us\n", best * 1e3);
    return 0;
}
