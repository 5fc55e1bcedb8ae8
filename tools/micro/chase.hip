// Micro-benchmark: dependent 64-B node loads (pointer chasing) in a table of
// `bytes`, every lane its own random chain; ns per step vs resident waves.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <random>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

struct alignas(64) Node { float4 a, b, c; int next[4]; };

__global__ __launch_bounds__(256) void k_chase(const Node* nodes, int steps, int* out, int nn)
{
    int cur = (int)((blockIdx.x * 256u + threadIdx.x) * 2654435761u % (unsigned)nn);
    float acc = 0;
    for (int s = 0; s < steps; s++) {
        const Node n = nodes[cur];
        acc += n.a.x + n.b.y + n.c.z;
        cur = n.next[s & 3];
    }
    out[blockIdx.x * 256 + threadIdx.x] = cur + (acc == 12345.f);
}

int main()
{
    for (size_t bytes : {(size_t)4 << 20, (size_t)32 << 20, (size_t)128 << 20, (size_t)1024 << 20}) {
        const int nn = (int)(bytes / 64);
        std::vector<Node> h(nn);
        std::mt19937 rng(1);
        for (int i = 0; i < nn; i++) {
            h[i].a = h[i].b = h[i].c = make_float4(1, 1, 1, 1);
            for (int k = 0; k < 4; k++) h[i].next[k] = (int)(rng() % nn);
        }
        Node* d;
        int* out;
        CHK(hipMalloc(&d, bytes));
        CHK(hipMalloc(&out, 8192 * 256 * 4));
        CHK(hipMemcpy(d, h.data(), bytes, hipMemcpyHostToDevice));
        hipEvent_t a, b;
        CHK(hipEventCreate(&a));
        CHK(hipEventCreate(&b));
        for (int grid : {256, 1024, 2048, 4096, 6144}) {
            const int steps = 200;
            float best = 1e9;
            for (int rep = 0; rep < 5; rep++) {
                CHK(hipEventRecord(a));
                hipLaunchKernelGGL(k_chase, dim3(grid), dim3(256), 0, 0, d, steps, out, nn);
                CHK(hipEventRecord(b));
                CHK(hipEventSynchronize(b));
                float ms;
                CHK(hipEventElapsedTime(&ms, a, b));
                if (ms < best) best = ms;
            }
            const double loads = (double)grid * 256 * steps;
            printf("table %5zu MB grid %5d: %7.1f ns/step  %6.2f Gloads/s  %7.1f GB/s (64B)\n", bytes >> 20, grid,
                   best * 1e6 / steps, loads / (best * 1e-3) / 1e9, loads * 64 / (best * 1e-3) / 1e9);
        }
        CHK(hipFree(d));
        CHK(hipFree(out));
    }
    return 0;
}
