// membench -- random 64-byte-block gather bandwidth and latency on one MI355X.
//
// The measured denominator SURVEY §8d asks for next to the 8 TB/s spec peak: the
// rank kernel's memory pattern is uniformly random 64-byte blocks over a ~2 GB
// table.  Modes:
//   indep  : every lane keeps D independent random 64-byte loads in flight
//   chain  : every lane follows a dependent chain (next address from the data)
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o tools/membench
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int D>
__global__ void k_indep(const uint4 *__restrict__ buf, uint64_t nblk, int iters, uint32_t *out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    uint64_t s = mix(gid + 1);
    for (int it = 0; it < iters; ++it) {
        uint4 v[D][4];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            s = mix(s + d);
            const uint4 *p = buf + (s % nblk) * 4;
            v[d][0] = p[0]; v[d][1] = p[1]; v[d][2] = p[2]; v[d][3] = p[3];
        }
#pragma unroll
        for (int d = 0; d < D; ++d)
            acc += v[d][0].x ^ v[d][1].y ^ v[d][2].z ^ v[d][3].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_chain(const uint4 *__restrict__ buf, uint64_t nblk, int iters, uint32_t *out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t b = mix(gid + 7) % nblk;
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const uint4 *p = buf + b * 4;
        uint4 a = p[0], c = p[1], d = p[2], e = p[3];
        acc += a.x ^ c.y ^ d.z ^ e.w;
        b = mix(b ^ a.x ^ e.w) % nblk;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint32_t *buf, uint64_t n)
{
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i < n; i += (uint64_t)gridDim.x * blockDim.x) buf[i] = (uint32_t)mix(i);
}

int main(int argc, char **argv)
{
    size_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : (size_t)2 << 30;
    int waves_per_cu = argc > 2 ? atoi(argv[2]) : 16;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    uint4 *buf; uint32_t *out;
    CHECK(hipMalloc(&buf, bytes));
    CHECK(hipMalloc(&out, 64));
    k_fill<<<4096, 256>>>((uint32_t *)buf, bytes / 4);
    CHECK(hipDeviceSynchronize());
    const uint64_t nblk = bytes / 64;
    const int blocks = prop.multiProcessorCount * waves_per_cu / 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    auto run = [&](const char *name, int D, int iters, auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        double loads = (double)blocks * 256 * iters * D;
        printf("{\"mode\": \"%s\", \"table_bytes\": %zu, \"waves_per_cu\": %d, \"inflight_per_lane\": %d, "
               "\"GBps\": %.1f, \"ns_per_load_per_lane\": %.1f}\n",
               name, bytes, waves_per_cu, D, loads * 64 / (ms * 1e-3) / 1e9, ms * 1e6 / (iters * (double)D));
    };
    const int it = 2000;
    run("indep", 1, it, [&] { k_indep<1><<<blocks, 256>>>(buf, nblk, it, out); });
    run("indep", 2, it / 2, [&] { k_indep<2><<<blocks, 256>>>(buf, nblk, it / 2, out); });
    run("indep", 4, it / 4, [&] { k_indep<4><<<blocks, 256>>>(buf, nblk, it / 4, out); });
    run("indep", 8, it / 8, [&] { k_indep<8><<<blocks, 256>>>(buf, nblk, it / 8, out); });
    run("chain", 1, it / 4, [&] { k_chain<<<blocks, 256>>>(buf, nblk, it / 4, out); });
    return 0;
}
