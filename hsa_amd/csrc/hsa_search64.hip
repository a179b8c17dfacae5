// hsa_search64.hip -- the 64-bit interval instantiation of the search (config 5: texts
// of 2^32 characters or more, which the reference's 32-bit bwtint_t cannot index,
// 2BWT-Interface.h:26).  The same kernels as hsa_search.hip (hsa_search_kernels.h),
// instantiated with IT = uint64_t: the same 16-byte rank blocks, counts modulo 2^32,
// with the index's count-wrap table for the high words (RankDir64, hsa_device.h),
// 32-byte stack entries, hsa_aln64_t hit records.
#include "hsa_search_kernels.h"

extern "C" int hsa_search_device64(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes,
                                   const hsa_device_batch_t *b, void *stream)
{
    return search_device_impl<uint64_t>(ix, regimes, n_regimes, b, stream);
}
