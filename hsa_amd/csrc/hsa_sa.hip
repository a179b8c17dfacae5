// hsa_sa.hip -- SA index -> text position, batched.
//
// One lane per SA index (the walk and the block search: hsa_sa.h).
#include <hip/hip_runtime.h>
#include <string.h>

#include "hsa_device.h"
#include "hsa_internal.h"
#include "hsa_sa.h"

struct SaArgs {
    SaView v;
    const uint32_t *idx;
    uint32_t *out;                 // 4 u32 per index: sa value, seq id, 1-based position, packed position
    size_t n;
};

__global__ void __launch_bounds__(256) k_sa_position(SaArgs a)
{
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    const uint32_t occ = hsa_sa_value(a.v, a.idx[t]);
    uint32_t sid = 0xffffffffu, ori = 0xffffffffu;
    hsa_sa_block(a.v, occ, sid, ori);
    reinterpret_cast<uint4 *>(a.out)[t] = make_uint4(occ, sid, ori, occ);
}

SaView hsa_sa_view(const hsa_index *ix)
{
    SaView v;
    v.blk = ix->blk[0]; v.isa0 = ix->isa0;
    memcpy(v.C, ix->C, sizeof v.C);
    v.sa = ix->d_sa; v.interval = ix->sa_interval; v.blocks = ix->d_blocks; v.n_blocks = ix->n_blocks;
    return v;
}

extern "C" int hsa_index_set_sa(hsa_index_t *ix, const uint32_t *sa_values, uint64_t n_values, uint32_t interval,
                                const uint32_t *blocks, int n_blocks)
{
    if (!sa_values || interval == 0 || n_values == 0 || n_blocks < 0 || (n_blocks && !blocks)) {
        hsa_set_error("hsa_index_set_sa: bad arguments");
        return HSA_E_ARG;
    }
    if (int rc0 = hsa_need32(ix)) return rc0;
    if (int rc0 = hsa_need_unshared(ix, "hsa_index_set_sa")) return rc0;
    if (n_values < ((uint64_t)ix->T + interval) / interval) {
        hsa_set_error("hsa_index_set_sa: %llu values < (T + s) / s", (unsigned long long)n_values);
        return HSA_E_ARG;
    }
    HSA_HIP(hipSetDevice(ix->device));
    (void)hipFree(ix->d_sa); (void)hipFree(ix->d_blocks);
    ix->d_sa = nullptr; ix->d_blocks = nullptr;
    if (hipMalloc(&ix->d_sa, n_values * 4) != hipSuccess ||
        hipMalloc(&ix->d_blocks, (size_t)(n_blocks ? n_blocks : 1) * 16) != hipSuccess) {
        hsa_set_error("hsa_index_set_sa: hipMalloc failed");
        return HSA_E_MEM;
    }
    HSA_HIP(hipMemcpy(ix->d_sa, sa_values, n_values * 4, hipMemcpyHostToDevice));
    if (n_blocks) HSA_HIP(hipMemcpy(ix->d_blocks, blocks, (size_t)n_blocks * 16, hipMemcpyHostToDevice));
    ix->sa_interval = interval;
    ix->n_blocks = (uint32_t)n_blocks;
    return 0;
}

extern "C" int hsa_sa_position_device(hsa_index_t *ix, size_t n, const uint32_t *d_idx, uint32_t *d_out4, void *stream)
{
    if (!ix->d_sa) { hsa_set_error("no suffix array attached (hsa_index_set_sa)"); return HSA_E_ARG; }
    HSA_HIP(hipSetDevice(ix->device));
    SaArgs A;
    A.v = hsa_sa_view(ix);
    A.idx = d_idx; A.out = d_out4; A.n = n;
    hipStream_t st = stream ? (hipStream_t)stream : ix->stream;
    if (n) hipLaunchKernelGGL(k_sa_position, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, A);
    HSA_HIP(hipGetLastError());
    return 0;
}

extern "C" int hsa_sa_position_batch(hsa_index_t *ix, size_t n, const uint32_t *sa_index, uint32_t *out4)
{
    int rc;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, n * 4 + 64)) || (rc = hsa_grow(&ix->d_out, &ix->d_out_cap, n * 16 + 64)))
        return rc;
    ix->staged_valid = 0;                      // d_in no longer holds the staged regimes
    HSA_HIP(hipSetDevice(ix->device));
    HSA_HIP(hipMemcpyAsync(ix->d_in, sa_index, n * 4, hipMemcpyHostToDevice, ix->stream));
    if ((rc = hsa_sa_position_device(ix, n, (const uint32_t *)ix->d_in, (uint32_t *)ix->d_out, ix->stream))) return rc;
    HSA_HIP(hipMemcpyAsync(out4, ix->d_out, n * 16, hipMemcpyDeviceToHost, ix->stream));
    HSA_HIP(hipStreamSynchronize(ix->stream));
    return 0;
}

