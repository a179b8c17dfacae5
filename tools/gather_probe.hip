// gather_probe -- what a random 64-byte-sector gather costs on one MI355X, by access
// shape.  The rank queries of the search kernels are uniformly random sectors of a
// table of 0.75-12 GB; this sweeps the shapes a kernel can choose between:
//   lane16   : each lane loads 16 B of its own random sector (64 sectors per wave load)
//   lane4    : each lane loads 4 B of its own random sector
//   coop4x16 : 4 adjacent lanes load the 4 x 16 B of one random sector (16 sectors per
//              wave load, every byte of the sector used)
//   lane64   : each lane loads its whole sector in four 16-B loads
//   chain16  : lane16, but the next sector depends on the loaded data (latency bound)
// Table sizes from Infinity-Cache resident to 3x the hg19-sized rank index; 8/16/32
// waves per CU; D independent loads in flight per lane.
// Output: one JSON line per run: sectors/s and GB/s of whole 64-B sectors touched.
// Build: hipcc -O3 --offload-arch=gfx950 tools/gather_probe.hip -o tools/gather_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ uint64_t mix(uint64_t z)
{
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// MODE 0 lane16, 1 lane4, 2 coop4x16, 3 lane64
template <int MODE, int D>
__global__ void __launch_bounds__(256) k_indep(const uint4 *__restrict__ buf, uint64_t nsec, int iters, uint32_t *out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t acc = 0;
    // coop: the 4 lanes of a group share the random stream
    uint64_t s = mix((MODE == 2 ? (gid >> 2) : gid) + 1);
    for (int it = 0; it < iters; ++it) {
        uint32_t v[D];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            s = mix(s + (uint64_t)d);
            const uint64_t sec = s % nsec;
            if (MODE == 0) {
                const uint4 q = buf[sec * 4 + (s >> 62)];
                v[d] = q.x ^ q.w;
            } else if (MODE == 1) {
                v[d] = reinterpret_cast<const uint32_t *>(buf)[sec * 16 + (s >> 60)];
            } else if (MODE == 2) {
                const uint4 q = buf[sec * 4 + (lane & 3u)];
                v[d] = q.x ^ q.w;
            } else {
                const uint4 *p = buf + sec * 4;
                const uint4 a = p[0], b = p[1], c = p[2], e = p[3];
                v[d] = a.x ^ b.y ^ c.z ^ e.w;
            }
        }
#pragma unroll
        for (int d = 0; d < D; ++d) acc += v[d];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(256) k_chain16(const uint4 *__restrict__ buf, uint64_t nsec, int iters, uint32_t *out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t s = mix(gid + 7);
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        const uint4 q = buf[(s % nsec) * 4 + (s >> 62)];
        acc += q.x;
        s = mix(s ^ q.y ^ q.w);
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// A wave-instruction with only `act` of its 64 lanes active: what a load costs the CU
// when few lanes of a divergent persistent kernel need it (each active lane 16 B of
// its own random sector).
__global__ void __launch_bounds__(256) k_sparse(const uint4 *__restrict__ buf, uint64_t nsec, int iters, int act,
                                                uint32_t *out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t acc = 0;
    uint64_t s = mix(gid + 1);
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        if (lane < (uint32_t)act) {
            const uint4 q = buf[(s % nsec) * 4 + (s >> 62)];
            acc += q.x ^ q.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// LDS-DMA rows: each active lane copies `words` dwords of its own random 128-byte row
// into LDS (global_load_lds_dword, one instruction per word), as k_search's strand start
__global__ void __launch_bounds__(256) k_dma(const uint32_t *__restrict__ buf, uint64_t nrows, int iters, int act,
                                             int words, uint32_t *out)
{
    __shared__ uint32_t lds[32 * 256];
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    uint64_t s = mix(gid + 1);
    uint32_t acc = 0;
    for (int it = 0; it < iters; ++it) {
        s = mix(s);
        if (lane < (uint32_t)act) {
            const uint32_t *src = buf + (s % nrows) * 32;
            uint32_t *dst = lds + (threadIdx.x & ~63u);
            for (int q = 0; q < words; ++q) __builtin_amdgcn_global_load_lds(src + q, dst + q * 256, 4, 0, 0);
            __builtin_amdgcn_s_waitcnt(0);
            acc += lds[threadIdx.x];
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_fill(uint32_t *buf, uint64_t n)
{
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        buf[i] = (uint32_t)mix(i);
}

int main(int argc, char **argv)
{
    const char *only = argc > 1 ? argv[1] : "";
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int n_cu = prop.multiProcessorCount;
    const size_t max_bytes = (size_t)12 << 30;
    uint4 *buf; uint32_t *out;
    CHECK(hipMalloc(&buf, max_bytes));
    CHECK(hipMalloc(&out, 64));
    k_fill<<<8192, 256>>>((uint32_t *)buf, max_bytes / 4);
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    if (!strcmp(only, "sparse")) {
        // loads per second by active lanes per wave instruction, 3 GB table, 16 waves/CU
        const size_t bytes = (size_t)3 << 30;
        const uint64_t nsec = bytes / 64;
        for (int act : {1, 2, 4, 8, 16, 32, 64}) {
            const int blocks = n_cu * 4, iters = 256;
            k_sparse<<<blocks, 256>>>(buf, nsec, iters / 4, act, out);
            CHECK(hipDeviceSynchronize());
            CHECK(hipEventRecord(e0));
            k_sparse<<<blocks, 256>>>(buf, nsec, iters, act, out);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double insts = (double)blocks * 4 * iters, lanes = insts * act;
            printf("{\"mode\": \"sparse\", \"active_lanes\": %d, \"Ginst_per_s\": %.3f, \"Glane_loads_per_s\": %.2f, "
                   "\"ns_per_inst_per_cu\": %.2f}\n", act, insts / (ms * 1e-3) / 1e9, lanes / (ms * 1e-3) / 1e9,
                   ms * 1e6 / (insts / n_cu));
        }
        for (int act : {1, 4, 16, 64}) {
            for (int words : {9, 26}) {
                const int blocks = n_cu * 4, iters = 64;
                k_dma<<<blocks, 256>>>((const uint32_t *)buf, bytes / 128, iters / 4, act, words, out);
                CHECK(hipDeviceSynchronize());
                CHECK(hipEventRecord(e0));
                k_dma<<<blocks, 256>>>((const uint32_t *)buf, bytes / 128, iters, act, words, out);
                CHECK(hipEventRecord(e1));
                CHECK(hipEventSynchronize(e1));
                float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
                const double rows = (double)blocks * 4 * iters * act, insts = (double)blocks * 4 * iters * words;
                printf("{\"mode\": \"dma\", \"active_lanes\": %d, \"words\": %d, \"Grows_per_s\": %.3f, "
                       "\"Ginst_per_s\": %.3f}\n", act, words, rows / (ms * 1e-3) / 1e9, insts / (ms * 1e-3) / 1e9);
            }
        }
        return 0;
    }
    const size_t sizes[] = {(size_t)128 << 20, (size_t)2 << 30, (size_t)6 << 30, (size_t)12 << 30};
    const int waves[] = {8, 16, 32};
    // lanes per sector and sectors per lane-load for the sector count
    auto run = [&](const char *name, size_t bytes, int wpc, int D, double sectors_per_lane_load, auto launch) {
        const int blocks = n_cu * wpc / 4;
        const int iters = 256;
        launch(blocks, iters / 4);
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        launch(blocks, iters);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        const double sectors = (double)blocks * 256 * iters * D * sectors_per_lane_load;
        printf("{\"mode\": \"%s\", \"table_bytes\": %zu, \"waves_per_cu\": %d, \"inflight_per_lane\": %d, "
               "\"Gsectors_per_s\": %.2f, \"GBps_of_sectors\": %.1f}\n",
               name, bytes, wpc, D, sectors / (ms * 1e-3) / 1e9, sectors * 64 / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    for (size_t bytes : sizes) {
        const uint64_t nsec = bytes / 64;
        for (int w : waves) {
            if (!*only || !strcmp(only, "lane16")) {
                run("lane16", bytes, w, 1, 1.0, [&](int b, int it) { k_indep<0, 1><<<b, 256>>>(buf, nsec, it, out); });
                run("lane16", bytes, w, 4, 1.0, [&](int b, int it) { k_indep<0, 4><<<b, 256>>>(buf, nsec, it, out); });
            }
            if (!*only || !strcmp(only, "lane4"))
                run("lane4", bytes, w, 4, 1.0, [&](int b, int it) { k_indep<1, 4><<<b, 256>>>(buf, nsec, it, out); });
            if (!*only || !strcmp(only, "coop4x16")) {
                run("coop4x16", bytes, w, 1, 0.25, [&](int b, int it) { k_indep<2, 1><<<b, 256>>>(buf, nsec, it, out); });
                run("coop4x16", bytes, w, 4, 0.25, [&](int b, int it) { k_indep<2, 4><<<b, 256>>>(buf, nsec, it, out); });
            }
            if (!*only || !strcmp(only, "lane64"))
                run("lane64", bytes, w, 2, 1.0, [&](int b, int it) { k_indep<3, 2><<<b, 256>>>(buf, nsec, it, out); });
            if (!*only || !strcmp(only, "chain16"))
                run("chain16", bytes, w, 1, 1.0, [&](int b, int it) { k_chain16<<<b, 256>>>(buf, nsec, it, out); });
        }
    }
    CHECK(hipFree(buf));
    return 0;
}
