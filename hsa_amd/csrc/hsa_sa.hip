// hsa_sa.hip -- SA index -> text position, batched.
//
// BWTSaValue (BWT.c:1195-1220) walks LF (BWTPsiMinusValue, BWT.c:1142-1162, via
// BWTOccValueOnSpot, BWT.c:924-959) until the SA index is a multiple of the
// sampling interval, then adds the steps to the sampled value;
// BWTRetrievePositionFromSAIndex (2BWT-Interface.c:329-361) then binary-searches the
// chromosome block table for (chrID, 1-based position).  Here one lane per SA index;
// every LF step is one 16-byte rank-block load (the character before the position and
// its count come from the same block), then one load of the sampled value.
#include <hip/hip_runtime.h>
#include <string.h>

#include "hsa_device.h"
#include "hsa_internal.h"

struct SaArgs {
    const uint4 *blk;
    uint32_t isa0;
    uint32_t C[4];
    const uint32_t *sa;            // sampled values; sa[0] = -1 as BWTLoad leaves it (BWT.c:222)
    uint32_t interval;
    const uint32_t *blocks;        // n_blocks rows (chrID, blockStart, blockEnd, ori), HSP.h:41-46
    uint32_t n_blocks;
    const uint32_t *idx;
    uint32_t *out;                 // 4 u32 per index: sa value, seq id, 1-based position, packed position
    size_t n;
};

// BWTPsiMinusValue: the LF map of SA index `index` (index != inverseSa0).
__device__ __forceinline__ uint32_t psi_minus(const SaArgs &a, uint32_t index)
{
    uint32_t i = index + 1u;
    i -= (i > a.isa0);                         // BWTOccValueOnSpot: '$' is not encoded (BWT.c:949)
    const uint32_t p = i - 1u;                 // the BWT character before i ...
    const uint4 q = a.blk[p >> 4];
    const uint32_t r = p & 15u;
    const uint32_t c = (q.w >> (2u * r)) & 3u;
    const uint32_t x = q.w ^ ~(c * 0x55555555u);
    const uint32_t n = __popc(x & (x >> 1) & 0x55555555u & ((1u << (2u * r)) - 1u));
    const uint32_t base = hsa_sel4(c, q.x, q.y, q.z, (p & ~15u) - q.x - q.y - q.z);
    const uint32_t cc = hsa_sel4(c, a.C[0], a.C[1], a.C[2], a.C[3]);
    return cc + base + n + 1u;                 // ... and its count up to and including it
}

__global__ void __launch_bounds__(256) k_sa_position(SaArgs a)
{
    const size_t t = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= a.n) return;
    uint32_t index = a.idx[t];
    uint32_t skipped = 0;
    while (index % a.interval != 0) {          // BWTSaValue
        ++skipped;
        index = index == a.isa0 ? 0u : psi_minus(a, index);
    }
    const uint32_t occ = a.sa[index / a.interval] + skipped;
    // the reference's binary search (h starts at nblock; see oracle/hsa_oracle.c for
    // the one case where it would read past the table: stopped as "not found")
    uint32_t sid = 0xffffffffu, ori = 0xffffffffu;
    uint32_t l = 0, h = a.n_blocks;
    while (l <= h) {
        const uint32_t m = (h + l) >> 1;
        if (m >= a.n_blocks) break;
        const uint32_t start = a.blocks[4 * m + 1];
        if (start > occ) { h = m - 1u; continue; }
        const uint32_t end = a.blocks[4 * m + 2];
        if (end < occ) { l = m + 1u; continue; }
        sid = a.blocks[4 * m];
        ori = occ - start + a.blocks[4 * m + 3] + 1u;
        break;
    }
    uint4 o = make_uint4(occ, sid, ori, occ);
    reinterpret_cast<uint4 *>(a.out)[t] = o;
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
    A.blk = ix->blk[0]; A.isa0 = ix->isa0;
    memcpy(A.C, ix->C, sizeof A.C);
    A.sa = ix->d_sa; A.interval = ix->sa_interval; A.blocks = ix->d_blocks; A.n_blocks = ix->n_blocks;
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

