// Micro-benchmark: the cost of a dependent kernel launch on one stream (the wavefront loop's
// k_trace -> k_step -> k_trace chain in its sparse phase), measured as the time per launch of
// a chain of N small kernels that each read the previous one's output:
//   stream   plain hipLaunchKernelGGL on one stream
//   graph    the same chain captured once into a hipGraph and launched as one graph
//   persist  one kernel doing N phases behind a grid barrier (an atomic counter per phase,
//            release/acquire at agent scope), grid no larger than the co-resident capacity
// with blocks x 256 threads each writing `bytes_per_thread` (dirty lines for the kernel-end
// release to write back).  Usage: launch_gap [blocks] [N] [bytes_per_thread]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#define CHK(x)                                                              \
    do {                                                                    \
        hipError_t e = (x);                                                 \
        if (e != hipSuccess) {                                              \
            printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            return 1;                                                       \
        }                                                                   \
    } while (0)

__global__ __launch_bounds__(256) void k_phase(const float* __restrict__ in, float* __restrict__ out, int words)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    float acc = in[(t * 7) % (gridDim.x * 256)];
    for (int w = 0; w < words; w++) out[(size_t)w * gridDim.x * 256 + t] = acc + (float)w;
}

// N phases in one launch; phase k reads buffer k&1 and writes buffer (k&1)^1, then every block
// arrives at counter k and waits until all have (bounded spin: a timeout sets *err and exits)
__global__ __launch_bounds__(256) void k_persist(float* a, float* b, int words, int n, unsigned* bar, int* err)
{
    const int t = blockIdx.x * 256 + threadIdx.x;
    const unsigned nb = gridDim.x;
    for (int k = 0; k < n; k++) {
        const float* in = (k & 1) ? b : a;
        float* out = (k & 1) ? a : b;
        float acc = in[(t * 7) % (gridDim.x * 256)];
        for (int w = 0; w < words; w++) out[(size_t)w * gridDim.x * 256 + t] = acc + (float)w;
        __syncthreads();
        if (threadIdx.x == 0) {
            __atomic_fetch_add(bar + k, 1u, __ATOMIC_RELEASE);
            long long spins = 0;
            while (__hip_atomic_load(bar + k, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < nb) {
                __builtin_amdgcn_s_sleep(1);
                if (++spins > (1ll << 24)) {
                    atomicExch(err, 1);
                    break;
                }
            }
        }
        __syncthreads();
        if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    }
}

int main(int argc, char** argv)
{
    int blocks = argc > 1 ? atoi(argv[1]) : 64;
    const int n = argc > 2 ? atoi(argv[2]) : 2000;
    const int bpt = argc > 3 ? atoi(argv[3]) : 16;
    const int words = bpt / 4;
    int dev_cus = 0;
    CHK(hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, 0));
    int per_cu = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(k_persist), 256, 0));
    const int cap = per_cu * dev_cus;
    const size_t elems = (size_t)blocks * 256 * (words > 0 ? words : 1);
    float *a, *b;
    unsigned* bar;
    int* err;
    CHK(hipMalloc(&a, elems * 4));
    CHK(hipMalloc(&b, elems * 4));
    CHK(hipMalloc(&bar, (size_t)n * 4));
    CHK(hipMalloc(&err, 4));
    CHK(hipMemset(a, 0, elems * 4));
    CHK(hipMemset(b, 0, elems * 4));
    hipStream_t s;
    CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    float ms = 0;
    // stream
    for (int rep = 0; rep < 2; rep++) {
        CHK(hipEventRecord(e0, s));
        for (int k = 0; k < n; k++)
            hipLaunchKernelGGL(k_phase, dim3(blocks), dim3(256), 0, s, (k & 1) ? b : a, (k & 1) ? a : b, words);
        CHK(hipEventRecord(e1, s));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("{\"blocks\": %d, \"n\": %d, \"bytes_per_thread\": %d, \"coresident_cap\": %d, \"stream_us\": %.2f", blocks, n,
           bpt, cap, ms * 1e3 / n);
    // graph (chains of 8, the host's batch, and of n)
    for (int chain : {8, n}) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int k = 0; k < chain; k++)
            hipLaunchKernelGGL(k_phase, dim3(blocks), dim3(256), 0, s, (k & 1) ? b : a, (k & 1) ? a : b, words);
        CHK(hipStreamEndCapture(s, &g));
        CHK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipEventRecord(e0, s));
            for (int k = 0; k < n / chain; k++) CHK(hipGraphLaunch(ge, s));
            CHK(hipEventRecord(e1, s));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
        }
        printf(", \"graph%d_us\": %.2f", chain, ms * 1e3 / ((n / chain) * chain));
        CHK(hipGraphExecDestroy(ge));
        CHK(hipGraphDestroy(g));
    }
    // persistent (only when the grid fits co-resident)
    if (blocks <= cap) {
        for (int rep = 0; rep < 2; rep++) {
            CHK(hipMemsetAsync(bar, 0, (size_t)n * 4, s));
            CHK(hipMemsetAsync(err, 0, 4, s));
            CHK(hipEventRecord(e0, s));
            hipLaunchKernelGGL(k_persist, dim3(blocks), dim3(256), 0, s, a, b, words, n, bar, err);
            CHK(hipEventRecord(e1, s));
            CHK(hipEventSynchronize(e1));
            CHK(hipEventElapsedTime(&ms, e0, e1));
        }
        int h_err = 0;
        CHK(hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost));
        printf(", \"persist_us\": %.2f, \"persist_timeout\": %d", ms * 1e3 / n, h_err);
    }
    // the kernel alone (one launch, long chain of its body): its own duration
    printf("}\n");
    return 0;
}
