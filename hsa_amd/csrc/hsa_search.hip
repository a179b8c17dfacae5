// hsa_search.hip -- the 32-bit search API (include/hsa_gpu.h): host-array and
// device-resident batches, direct bwt_match_gap calls, the splice seeds; the kernels
// are in hsa_search_kernels.h.
#include "hsa_search_kernels.h"

#include <vector>

// ---------------------------------------------------------------- splice seeds
// The seed calls of bwt_splice_match (bwtgap.c:797-812) for every read the main pass
// flagged HSA_F_FALLBACK: one thread per (read, strand).  The strand's three seeds
// t = 0, 1, 2 (sl = len / 3, la_t = sl + (t == 2 ? len % 3 : 0)) search [t sl, t sl +
// la_t) of the strand sequence with the widths of its PREFIX of length la_t
// (bwtgap.c:807-809; bwt_cal_width type 1, bwtaln.c:84-97: forward extension on the
// reverse BWT).  The three prefixes share their first sl positions, so one chain over
// la_2 characters fills all three width slots; each slot ends with its own terminal
// {0, bid + 1} (bwtaln.c:113-114).
struct SeedArgs {
    RankDir rev;
    uint32_t T;
    uint32_t C[5];
    const hsa_job_t *rjobs;
    const uint8_t *rcodes;
    const uint32_t *rflags;
    uint32_t n_reads;
    int32_t max_seed_diff;
    uint32_t code_stride, pair_stride;   // per read: seed codes (bytes), width pairs
    hsa_job_t *jobs;
    hsa_mg_job_t *mg;
    uint8_t *codes;
    int32_t *cw;
    int32_t *list;
    unsigned long long *count;
    unsigned long long *ctr;
};

__global__ void __launch_bounds__(BLOCK) k_seed_prep(SeedArgs a)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t r = t >> 1, s = t & 1u;
    if (r >= a.n_reads || !(a.rflags[r] & HSA_F_FALLBACK)) return;
    const hsa_job_t R = a.rjobs[r];
    const uint32_t L = R.len, sl = L / 3u;
    if (sl < 1) return;
    const uint32_t la2 = sl + L % 3u;
    auto base = [&](uint32_t p) -> uint32_t {          // strand s, position p
        const uint32_t c = a.rcodes[R.off + (s ? L - 1u - p : p)];
        return s && c < 4 ? 3u - c : c;
    };
    // call i = 3 s + tt of read r: codes and width pairs at fixed offsets in the read's slots
    uint32_t coff[3], poff[3], la[3];
    {
        uint32_t co = 0, po = 0;
        for (uint32_t i = 0; i < 6; ++i) {
            const uint32_t l_i = sl + (i % 3 == 2 ? L % 3u : 0u);
            if (i / 3 == s) { coff[i % 3] = co; poff[i % 3] = po; la[i % 3] = l_i; }
            co += l_i; po += l_i + 1;
        }
    }
    uint8_t *const cbase = a.codes + (size_t)r * a.code_stride;
    int32_t *const wbase = a.cw + 2 * (size_t)r * a.pair_stride;
    uint32_t k = 0, l = a.T, bid = 0, bid_sl = 0, q = 0;
    for (uint32_t p = 0; p < la2; ++p) {
        const uint32_t c = base(p);
        if (c < 4) {
            uint32_t ok, ol;
            hsa_occ1_pair(a.rev, k, l + 1u, c, ok, ol);
            q += 2;
            const uint32_t cc = hsa_sel4(c, a.C[0], a.C[1], a.C[2], a.C[3]);
            k = cc + ok + 1u;
            l = cc + ol;
        }
        if (k > l || c > 3) { k = 0; l = a.T; ++bid; }
        const int32_t w = (int32_t)(l - k + 1u);
        for (uint32_t tt = 0; tt < 3; ++tt)
            if (p < la[tt]) { wbase[2 * (poff[tt] + p)] = w; wbase[2 * (poff[tt] + p) + 1] = (int32_t)bid; }
        if (p + 1 == sl) bid_sl = bid;
        // seed codes: strand position p belongs to seed tt = p / sl (the last seed runs to la2 + 2 sl)
    }
    for (uint32_t tt = 0; tt < 3; ++tt) {
        const uint32_t term_bid = (la[tt] == sl ? bid_sl : bid) + 1u;
        wbase[2 * (poff[tt] + la[tt])] = 0;
        wbase[2 * (poff[tt] + la[tt]) + 1] = (int32_t)term_bid;
        for (uint32_t p = 0; p < la[tt]; ++p) cbase[coff[tt] + p] = (uint8_t)base(tt * sl + p);
        const uint32_t j = r * 6u + 3u * s + tt;
        hsa_job_t J;
        J.off = (uint64_t)r * a.code_stride + coff[tt];
        J.len = la[tt];
        J.max_diff = a.max_seed_diff;
        J.seed_len = (int32_t)la[tt];
        J.regime = 0;
        a.jobs[j] = J;
        hsa_mg_job_t M;
        M.wb_off = (uint64_t)r * a.pair_stride + poff[tt];
        M.ws_off = 0;
        M.strand = (int32_t)s;
        M.seed = HSA_SEED_ALIAS;
        a.mg[j] = M;
    }
    const unsigned long long b0 = atomicAdd(a.count, 3ull);
    for (uint32_t tt = 0; tt < 3; ++tt) a.list[b0 + tt] = (int32_t)(r * 6u + 3u * s + tt);
    atomicAdd(&a.ctr[7], (unsigned long long)q);
}

// ---------------------------------------------------------------- host side
#ifdef HSA_DIAG
extern "C" int hsa_diag_read(unsigned long long *out, int n_blocks)
{
    HSA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_diag), sizeof(unsigned long long) * 4 * (size_t)n_blocks));
    return 0;
}
extern "C" int hsa_diag_counters(unsigned long long *out, int reset)
{
    HSA_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dctr), sizeof(unsigned long long) * 32));
    if (reset) {
        unsigned long long z[32] = {0};
        HSA_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_dctr), z, sizeof z));
    }
    return 0;
}
#endif
struct MgHost {
    const hsa_mg_job_t *mg;
    const int32_t *widths;
    size_t width_pairs;
    int32_t *widths_out;
};

// Checks of a caller-width batch; max_seed = the longest own width_seed.  A width_seed
// with seed_len > len makes the reference read outside it: refused.
static int mg_limits(const hsa_job_t *jobs, const hsa_mg_job_t *mg, int n, const MgHost &mh, int &max_seed)
{
    max_seed = 0;
    for (int j = 0; j < n; ++j) {
        const hsa_mg_job_t &M = mg[j];
        const uint32_t len = jobs[j].len;
        if (M.strand != 0 && M.strand != 1) { hsa_set_error("call %d: strand %d", j, M.strand); return HSA_E_ARG; }
        if (M.seed < HSA_SEED_NONE || M.seed > HSA_SEED_ALIAS) { hsa_set_error("call %d: seed kind", j); return HSA_E_ARG; }
        if (M.seed != HSA_SEED_NONE && (jobs[j].seed_len < 0 || jobs[j].seed_len > (int)len)) {
            hsa_set_error("call %d: width_seed with seed_len %d outside [0, len %u] (undefined in the reference)", j,
                          jobs[j].seed_len, len);
            return HSA_E_ARG;
        }
        if (M.wb_off + len + 1 > mh.width_pairs ||
            (M.seed == HSA_SEED_OWN && M.ws_off + (uint64_t)jobs[j].seed_len + 1 > mh.width_pairs)) {
            hsa_set_error("call %d: widths outside the width array", j);
            return HSA_E_ARG;
        }
        for (uint32_t t = 0; t <= len; ++t)
            if (mh.widths[2 * (M.wb_off + t) + 1] < 0) { hsa_set_error("call %d: negative bid", j); return HSA_E_ARG; }
        if (M.seed == HSA_SEED_OWN) {
            for (int t = 0; t <= jobs[j].seed_len; ++t)
                if (mh.widths[2 * (M.ws_off + t) + 1] < 0) { hsa_set_error("call %d: negative bid", j); return HSA_E_ARG; }
            if (jobs[j].seed_len > max_seed) max_seed = jobs[j].seed_len;
        }
    }
    return 0;
}

// k_search_any over host arrays (hsa_search_any.h): reads longer than k_search holds,
// or every read of a regime outside its layouts.  Same outputs as search_batch_impl.
static long search_any_host(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs, int n,
                            const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags, uint64_t *hit_off,
                            uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh)
{
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = ix->stream;
    uint32_t max_len = 1, max_seed = 0;
    for (int j = 0; j < n; ++j) {
        if (jobs[j].len > max_len) max_len = jobs[j].len;
        const bool own = mh ? mh->mg[j].seed == HSA_SEED_OWN : (int)jobs[j].len > jobs[j].seed_len;
        if (own && (uint32_t)jobs[j].seed_len > max_seed) max_seed = (uint32_t)jobs[j].seed_len;
    }
    AnyBufs AB;
    int rc = any_prepare(ix, regimes, n_regimes, (size_t)n, st, AB);
    if (rc) return rc;
    // inputs after the fast path's regime staging ([0, 1536) of d_in stays as it is)
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_jobs = 1536, o_codes = o_jobs + al((size_t)n * sizeof(hsa_job_t));
    const size_t o_mg = o_codes + al(codes_len + 64), o_cw = o_mg + (mh ? al((size_t)n * sizeof(hsa_mg_job_t)) : 0);
    const size_t cw_bytes = mh ? mh->width_pairs * 8 : 0;
    void *before = ix->d_in;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, o_cw + cw_bytes + 256))) return rc;
    if (before != ix->d_in) ix->staged_valid = 0;       // the regime staging went with the old buffer
    char *din = (char *)ix->d_in;
    HSA_HIP(hipMemcpyAsync(din + o_jobs, jobs, sizeof(hsa_job_t) * n, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(din + o_codes, codes, codes_len, hipMemcpyHostToDevice, st));
    MgPass mgp{nullptr, nullptr};
    if (mh) {
        HSA_HIP(hipMemcpyAsync(din + o_mg, mh->mg, sizeof(hsa_mg_job_t) * n, hipMemcpyHostToDevice, st));
        HSA_HIP(hipMemcpyAsync(din + o_cw, mh->widths, cw_bytes, hipMemcpyHostToDevice, st));
        mgp = MgPass{(const hsa_mg_job_t *)(din + o_mg), (int32_t *)(din + o_cw)};
    }
    const uint64_t hit_cap = (uint64_t)n * 64 + 65536;
    const size_t o_fl = al((size_t)n * 4), o_ho = o_fl + al((size_t)n * 4), o_hits = o_ho + al((size_t)n * 8);
    if ((rc = hsa_grow(&ix->d_out, &ix->d_out_cap, o_hits + hit_cap * 36 + 256))) return rc;
    char *dout = (char *)ix->d_out;
    unsigned long long *d_ctr = (unsigned long long *)ix->d_ctr;
    HSA_HIP(hipMemsetAsync(d_ctr, 0, 16 * sizeof(unsigned long long), st));
    HSA_HIP(hipEventRecord(ix->ev0, st));
    const hsa_job_t *dj = (const hsa_job_t *)(din + o_jobs);
    const uint8_t *dc = (const uint8_t *)(din + o_codes);
    int32_t *d_n = (int32_t *)dout;
    uint32_t *d_fl = (uint32_t *)(dout + o_fl);
    uint64_t *d_ho = (uint64_t *)(dout + o_ho);
    uint32_t *d_hits = (uint32_t *)(dout + o_hits);
    if ((rc = any_pass<uint32_t>(ix, AB, regimes, n_regimes, dj, nullptr, nullptr, n, (size_t)n, max_len, max_seed, dc,
                                 mh ? &mgp : nullptr, d_n, d_fl, d_ho, d_hits, hit_cap, d_ctr, AB.cnt + 2, AB.l_ovf,
                                 AB.cnt + 3, false, st)) ||
        (rc = any_pass<uint32_t>(ix, AB, regimes, n_regimes, dj, AB.l_ovf, AB.cnt + 3, 0, (size_t)n, max_len, max_seed,
                                 dc, mh ? &mgp : nullptr, d_n, d_fl, d_ho, d_hits, hit_cap, d_ctr, AB.cnt + 4, nullptr,
                                 nullptr, true, st)))
        return rc;
    HSA_HIP(hipEventRecord(ix->ev1, st));
    unsigned long long ctr[16];
    HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(n_aln, d_n, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(flags, d_fl, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(hit_off, d_ho, (size_t)n * 8, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    if (ctr[5]) { hsa_set_error("%llu reads pushed a score past the regime's n_stacks", ctr[5]); return HSA_E_ARG; }
    if (ctr[11]) { hsa_set_error("%llu reads exceed the large-pass capacity", ctr[11]); return HSA_E_ARG; }
    float ms = 0;
    HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
    const uint64_t total = ctr[1] < hit_cap ? ctr[1] : hit_cap;
    uint32_t *h = (uint32_t *)malloc((total + 1) * 36);
    if (!h) { hsa_set_error("host allocation of %llu hits failed", (unsigned long long)total); return HSA_E_MEM; }
    if (total) HSA_HIP(hipMemcpy(h, d_hits, total * 36, hipMemcpyDeviceToHost));
    if (mh) {
        int32_t *cw = (int32_t *)malloc(cw_bytes + 8);
        HSA_HIP(hipMemcpy(cw, din + o_cw, cw_bytes, hipMemcpyDeviceToHost));
        for (int j = 0; j < n; ++j)
            memcpy(mh->widths_out + 2 * mh->mg[j].wb_off, cw + 2 * mh->mg[j].wb_off, 8 * ((size_t)jobs[j].len + 1));
        free(cw);
    }
    if (stats) {
        stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
        stats->kernel_ms += ms; stats->main_kernel_ms += ms; stats->main_launches += 1;
    }
    *hits_out = h;
    return (long)total;
}

// A batch with reads (or a regime) k_search cannot hold: the reads it can hold through
// search_batch_impl, the others through k_search_any; outputs merged in job order.
static long search_batch_impl(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                              int n_jobs, const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                              uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh);

static long search_split(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs, int n,
                         const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags, uint64_t *hit_off,
                         uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh, bool fast_rg)
{
    std::vector<int> part[2];                        // 0: k_search, 1: k_search_any
    for (int j = 0; j < n; ++j) part[fast_rg && jobs[j].len <= FAST_MAX_LEN ? 0 : 1].push_back(j);
    uint32_t *hs[2] = {nullptr, nullptr};
    long tot[2] = {0, 0};
    if (stats) memset(stats, 0, sizeof *stats);
    for (int k = 0; k < 2; ++k) {
        const int m = (int)part[k].size();
        if (m == 0) continue;
        std::vector<hsa_job_t> pj(m);
        std::vector<hsa_mg_job_t> pm(mh ? m : 0);
        for (int q = 0; q < m; ++q) {
            pj[q] = jobs[part[k][q]];
            if (mh) pm[q] = mh->mg[part[k][q]];
        }
        const MgHost pmh = mh ? MgHost{pm.data(), mh->widths, mh->width_pairs, mh->widths_out} : MgHost{};
        std::vector<int32_t> na(m);
        std::vector<uint32_t> fl(m);
        std::vector<uint64_t> ho(m);
        hsa_stats_t ps;
        memset(&ps, 0, sizeof ps);
        const long t = k == 0 ? search_batch_impl(ix, regimes, n_regimes, pj.data(), m, codes, codes_len, na.data(), fl.data(),
                                                  ho.data(), &hs[k], &ps, mh ? &pmh : nullptr)
                              : search_any_host(ix, regimes, n_regimes, pj.data(), m, codes, codes_len, na.data(),
                                                fl.data(), ho.data(), &hs[k], &ps, mh ? &pmh : nullptr);
        if (t < 0) { free(hs[0]); free(hs[1]); return t; }
        tot[k] = t;
        for (int q = 0; q < m; ++q) {
            const int j = part[k][q];
            n_aln[j] = na[q]; flags[j] = fl[q]; hit_off[j] = ho[q] + (k ? (uint64_t)tot[0] : 0);
        }
        if (stats) {
            stats->rank_queries += ps.rank_queries; stats->blocks_loaded += ps.blocks_loaded; stats->pops += ps.pops;
            stats->overflow_reruns += ps.overflow_reruns; stats->kernel_ms += ps.kernel_ms;
            stats->main_kernel_ms += ps.main_kernel_ms; stats->main_launches += ps.main_launches;
        }
    }
    uint32_t *h = (uint32_t *)malloc(((size_t)tot[0] + (size_t)tot[1] + 1) * 36);
    if (tot[0]) memcpy(h, hs[0], (size_t)tot[0] * 36);
    if (tot[1]) memcpy(h + (size_t)tot[0] * 9, hs[1], (size_t)tot[1] * 36);
    free(hs[0]); free(hs[1]);
    *hits_out = h;
    return tot[0] + tot[1];
}

static long search_batch_impl(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                              int n_jobs, const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                              uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats, const MgHost *mh)
{
    *hits_out = nullptr;
    if (n_regimes < 1 || n_regimes > 2) { hsa_set_error("1 or 2 regimes"); return HSA_E_ARG; }
    if (int rc0 = hsa_need32(ix)) return rc0;
    int rc = check_regimes(regimes, n_regimes);
    if (rc) return rc;
    int max_len, max_seed;
    if ((rc = jobs_limits(jobs, n_jobs, max_len, max_seed))) return rc;
    if (mh && (rc = mg_limits(jobs, mh->mg, n_jobs, *mh, max_seed))) return rc;
    if (codes_len >= 0xFFFFFFFFull) { hsa_set_error("read codes of one call must be < 4 GiB"); return HSA_E_ARG; }
    HSA_HIP(hipSetDevice(ix->device));      // before any split: both halves allocate on ix's device
    for (int j = 0; j < n_jobs; ++j)        // the kernels read codes[off, off + len) of every job
        if (jobs[j].off > codes_len || jobs[j].len > codes_len - jobs[j].off) {
            hsa_set_error("job %d: codes [%llu, +%u) past codes_len %zu", j, (unsigned long long)jobs[j].off,
                          jobs[j].len, codes_len);
            return HSA_E_ARG;
        }
    {
        const bool fast_rg = fast_regimes(regimes, n_regimes);
        bool all_fit = fast_rg;
        for (int j = 0; j < n_jobs && all_fit; ++j) all_fit = jobs[j].len <= FAST_MAX_LEN;
        if (!all_fit)
            return search_split(ix, regimes, n_regimes, jobs, n_jobs, codes, codes_len, n_aln, flags, hit_off, hits_out,
                                stats, mh, fast_rg);
    }
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = ix->stream;
    if (stats) memset(stats, 0, sizeof *stats);
    if (n_jobs == 0) { *hits_out = (uint32_t *)calloc(9, 4); return 0; }
    static const bool verbose = getenv("HSA_VERBOSE") != nullptr;
    const auto now = []() { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; };
    const double tv0 = verbose ? now() : 0.0;

    // device staging: regimes+bmap | jobs | list | codes [| mg jobs | caller widths]
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_reg = 0, o_jobs = 1536, o_list = o_jobs + al((size_t)n_jobs * sizeof(hsa_job_t));
    const size_t o_codes = o_list + al((size_t)n_jobs * 4);
    const size_t o_mg = o_codes + al(codes_len + 1);
    const size_t o_cw = o_mg + (mh ? al((size_t)n_jobs * sizeof(hsa_mg_job_t)) : 0);
    const size_t cw_bytes = mh ? mh->width_pairs * 8 : 0;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, o_cw + cw_bytes + 256))) return rc;
    char *din = (char *)ix->d_in;
    int nb = 0;
    if ((rc = stage_regimes(ix, regimes, n_regimes, din + o_reg, nb, st, true))) return rc;
    const hsa_regime_t *d_reg = (const hsa_regime_t *)(din + o_reg);
    const uint8_t *d_bmap = (const uint8_t *)(din + o_reg + 256);
    HSA_HIP(hipMemcpyAsync(din + o_jobs, jobs, sizeof(hsa_job_t) * n_jobs, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(din + o_codes, codes, codes_len, hipMemcpyHostToDevice, st));
    MgPass mgp{nullptr, nullptr};
    if (mh) {
        HSA_HIP(hipMemcpyAsync(din + o_mg, mh->mg, sizeof(hsa_mg_job_t) * n_jobs, hipMemcpyHostToDevice, st));
        HSA_HIP(hipMemcpyAsync(din + o_cw, mh->widths, cw_bytes, hipMemcpyHostToDevice, st));
        mgp = MgPass{(const hsa_mg_job_t *)(din + o_mg), (int32_t *)(din + o_cw)};
    }
    const MgPass *mgpp = mh ? &mgp : nullptr;
    // outputs: n_aln | flags | hit_off | hits
    uint64_t hit_cap = (uint64_t)n_jobs * 4 + 4096;
    const size_t o_fl = ((size_t)n_jobs * 4 + 255) / 256 * 256;
    const size_t o_ho = o_fl + ((size_t)n_jobs * 4 + 255) / 256 * 256;
    const size_t o_hits = o_ho + ((size_t)n_jobs * 8 + 255) / 256 * 256;
    if ((rc = hsa_grow(&ix->d_out, &ix->d_out_cap, o_hits + hit_cap * 36 + 256))) return rc;
    char *dout = (char *)ix->d_out;
    int32_t *d_n = (int32_t *)dout;
    uint32_t *d_fl = (uint32_t *)(dout + o_fl);
    uint64_t *d_ho = (uint64_t *)(dout + o_ho);
    uint32_t *d_hits = (uint32_t *)(dout + o_hits);
    unsigned long long *d_ctr = (unsigned long long *)ix->d_ctr;

    LaunchPlan P;
    const bool gaps = any_gaps(regimes, n_regimes);
    const bool wide = need_wide(regimes, n_regimes);
    bool nib_ok = !mgpp && nib_exact(regimes, n_regimes);
    for (int j = 0; j < n_jobs && nib_ok; ++j) nib_ok = jobs[j].max_diff <= 6;
    if ((rc = plan_launch(ix, n_jobs, max_len, max_seed, nb, gaps, wide, PASS_MAIN, P, 0, 16, nib_ok))) return rc;
    HSA_HIP(hipEventRecord(ix->ev0, st));
    if ((rc = launch_pass(ix, P, ix->main, d_reg, d_bmap, (const hsa_job_t *)(din + o_jobs), nullptr, n_jobs,
                          max_len, max_seed, (const uint8_t *)(din + o_codes), d_n, d_fl, d_ho, d_hits, hit_cap, d_ctr, st,
                          nullptr, nullptr, 0, mgpp)))
        return rc;
    HSA_HIP(hipEventRecord(ix->ev1, st));
    unsigned long long ctr[8];
    HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(n_aln, d_n, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(flags, d_fl, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipMemcpyAsync(hit_off, d_ho, (size_t)n_jobs * 8, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    if (ctr[5]) { hsa_set_error("%llu reads exceed the regime's max_diff bound", ctr[5]); return HSA_E_ARG; }
    float ms = 0;
    HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
    uint64_t total = ctr[1] < hit_cap ? ctr[1] : hit_cap;
    const double tv1 = verbose ? now() : 0.0;
    uint32_t *h = (uint32_t *)malloc((total + 1) * 36);
    if (total) HSA_HIP(hipMemcpy(h, d_hits, total * 36, hipMemcpyDeviceToHost));
    if (verbose)
        fprintf(stderr, "[hsa] search of %d reads: copies in + kernels + result arrays out %.1f ms (kernels %.1f ms), "
                        "hits out %.1f ms\n", n_jobs, 1e3 * (tv1 - tv0), ms, 1e3 * (now() - tv1));
    if (stats) {
        stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
        stats->kernel_ms += ms; stats->main_kernel_ms += ms; stats->main_launches += 1;
    }

    // overflowed reads: re-run with large per-read capacity (never a CPU path)
    for (int round = 0; round < 4; ++round) {
        int32_t *list = (int32_t *)malloc(sizeof(int32_t) * n_jobs);
        int n_over = 0;
        for (int j = 0; j < n_jobs; ++j) if (flags[j] & HSA_F_OVERFLOW) list[n_over++] = j;
        if (n_over == 0) { free(list); break; }
        if (stats) stats->overflow_reruns += n_over;
        LaunchPlan B;
        int max_entries = 0;
        for (int r = 0; r < n_regimes; ++r) max_entries = regimes[r].max_entries > max_entries ? regimes[r].max_entries : max_entries;
        const int mode = round == 0 ? PASS_BIG : PASS_HUGE;
        if ((rc = plan_launch(ix, n_over, max_len, max_seed, nb, gaps, wide, mode, B, max_entries, 16, nib_ok))) {
            free(list); free(h); return rc;
        }
        uint64_t cap2 = (uint64_t)n_over * 256 * (round + 1) + 65536;
        void *d2 = nullptr;
        size_t o2_fl = ((size_t)n_jobs * 4 + 255) / 256 * 256;
        size_t o2_ho = o2_fl * 2, o2_hits = o2_ho + ((size_t)n_jobs * 8 + 255) / 256 * 256;
        HSA_HIP(hipMalloc(&d2, o2_hits + cap2 * 36));
        HSA_HIP(hipMemcpyAsync(din + o_list, list, sizeof(int32_t) * n_over, hipMemcpyHostToDevice, st));
        char *c2 = (char *)d2;
        HSA_HIP(hipEventRecord(ix->ev0, st));
        if ((rc = launch_pass(ix, B, mode == PASS_BIG ? ix->big : ix->huge, d_reg, d_bmap, (const hsa_job_t *)(din + o_jobs),
                              (const int32_t *)(din + o_list), n_over, max_len, max_seed,
                              (const uint8_t *)(din + o_codes), (int32_t *)c2,
                              (uint32_t *)(c2 + o2_fl), (uint64_t *)(c2 + o2_ho), (uint32_t *)(c2 + o2_hits), cap2,
                              d_ctr, st, nullptr, nullptr, 0, mgpp))) {
            free(list); free(h); (void)hipFree(d2); return rc;
        }
        HSA_HIP(hipEventRecord(ix->ev1, st));
        int32_t *n2 = (int32_t *)malloc((size_t)n_jobs * 4);
        uint32_t *f2 = (uint32_t *)malloc((size_t)n_jobs * 4);
        uint64_t *o2 = (uint64_t *)malloc((size_t)n_jobs * 8);
        HSA_HIP(hipMemcpyAsync(ctr, d_ctr, sizeof ctr, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(n2, c2, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(f2, c2 + o2_fl, (size_t)n_jobs * 4, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipMemcpyAsync(o2, c2 + o2_ho, (size_t)n_jobs * 8, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipStreamSynchronize(st));
        HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
        uint64_t t2 = ctr[1] < cap2 ? ctr[1] : cap2;
        h = (uint32_t *)realloc(h, (total + t2 + 1) * 36);
        if (t2) HSA_HIP(hipMemcpy(h + total * 9, c2 + o2_hits, t2 * 36, hipMemcpyDeviceToHost));
        for (int q = 0; q < n_over; ++q) {
            int j = list[q];
            n_aln[j] = n2[j]; flags[j] = f2[j]; hit_off[j] = o2[j] + total;
        }
        total += t2;
        if (stats) {
            stats->rank_queries += ctr[2]; stats->blocks_loaded += ctr[3]; stats->pops += ctr[4];
            stats->kernel_ms += ms;
        }
        free(n2); free(f2); free(o2); free(list);
        (void)hipFree(d2);
    }
    for (int j = 0; j < n_jobs; ++j)
        if (flags[j] & HSA_F_OVERFLOW) { hsa_set_error("read %d exceeds the large-pass capacity", j); free(h); return HSA_E_ARG; }
    if (mh) {
        // width_back of every call after its search (k_widths_export wrote them in place)
        int32_t *cw = (int32_t *)malloc(cw_bytes + 8);
        HSA_HIP(hipMemcpy(cw, din + o_cw, cw_bytes, hipMemcpyDeviceToHost));
        for (int j = 0; j < n_jobs; ++j)
            memcpy(mh->widths_out + 2 * mh->mg[j].wb_off, cw + 2 * mh->mg[j].wb_off, 8 * ((size_t)jobs[j].len + 1));
        free(cw);
    }
    *hits_out = h;
    return (long)total;
}

extern "C" long hsa_search_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                                 int n_jobs, const uint8_t *codes, size_t codes_len, int32_t *n_aln, uint32_t *flags,
                                 uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats)
{
    return search_batch_impl(ix, regimes, n_regimes, jobs, n_jobs, codes, codes_len, n_aln, flags, hit_off, hits_out,
                             stats, nullptr);
}

extern "C" long hsa_match_gap_batch(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes, const hsa_job_t *jobs,
                                    const hsa_mg_job_t *mg, int n_jobs, const uint8_t *codes, size_t codes_len,
                                    const int32_t *widths, size_t width_pairs, int32_t *widths_out, int32_t *n_aln,
                                    uint64_t *hit_off, uint32_t **hits_out, hsa_stats_t *stats)
{
    *hits_out = nullptr;
    if (n_jobs > 0 && (!mg || !widths || !widths_out)) { hsa_set_error("hsa_match_gap_batch: null argument"); return HSA_E_ARG; }
    uint32_t *flags = (uint32_t *)malloc(sizeof(uint32_t) * ((size_t)n_jobs + 1));
    const MgHost mh{mg, widths, width_pairs, widths_out};
    const long r = search_batch_impl(ix, regimes, n_regimes, jobs, n_jobs, codes, codes_len, n_aln, flags, hit_off,
                                     hits_out, stats, &mh);
    free(flags);
    return r;
}

extern "C" int hsa_search_device(hsa_index_t *ix, const hsa_regime_t *regimes, int n_regimes,
                                 const hsa_device_batch_t *b, void *stream)
{
    if (int rc = hsa_need32(ix)) return rc;
    return search_device_impl<uint32_t>(ix, regimes, n_regimes, b, stream);
}

extern "C" int hsa_splice_seeds_device(hsa_index_t *ix, const hsa_regime_t *seed_regime, const hsa_seed_batch_t *b,
                                       void *stream)
{
    if (int rc0 = hsa_need32(ix)) return rc0;
    int rc = check_regimes(seed_regime, 1);
    if (rc) return rc;
    if (seed_regime->max_gapo != 0) { hsa_set_error("seed searches have no gap opens (bwtgap.c:772)"); return HSA_E_ARG; }
    if (b->max_len < 3 || b->max_len > 1023 || b->n_jobs < 0) { hsa_set_error("max_len/n_jobs out of range"); return HSA_E_ARG; }
    const size_t n = (size_t)b->n_jobs, calls = 6 * n;
    if (n == 0) return 0;
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = stream ? (hipStream_t)stream : ix->stream;
    const uint32_t code_stride = (uint32_t)(2 * b->max_len), pair_stride = (uint32_t)(2 * b->max_len + 6);
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    const size_t o_mg = al(calls * sizeof(hsa_job_t)), o_list = o_mg + al(calls * sizeof(hsa_mg_job_t));
    const size_t o_fl = o_list + al(calls * 4), o_cnt = o_fl + al(calls * 4), o_codes = o_cnt + 256;
    const size_t o_cw = o_codes + al(n * code_stride), total = o_cw + n * pair_stride * 8 + 256;
    if ((rc = hsa_grow(&ix->d_seed, &ix->d_seed_cap, total))) return rc;
    char *d = (char *)ix->d_seed;
    unsigned long long *cnt = (unsigned long long *)(d + o_cnt);
    unsigned long long *ctr = (unsigned long long *)b->d_counters;
    HSA_HIP(hipMemsetAsync(cnt, 0, 8, st));
    SeedArgs S;
    S.rev = RankDir{ix->blk[1], ix->risa0};
    S.T = ix->T;
    memcpy(S.C, ix->C, sizeof S.C);
    S.rjobs = b->d_jobs; S.rcodes = b->d_codes; S.rflags = b->d_flags; S.n_reads = (uint32_t)n;
    S.max_seed_diff = seed_regime->max_diff;
    S.code_stride = code_stride; S.pair_stride = pair_stride;
    S.jobs = (hsa_job_t *)d; S.mg = (hsa_mg_job_t *)(d + o_mg); S.codes = (uint8_t *)(d + o_codes);
    S.cw = (int32_t *)(d + o_cw); S.list = (int32_t *)(d + o_list); S.count = cnt; S.ctr = ctr;
    // the search pass zeroes the counters first; the width queries are added after it
    void *before = ix->d_in;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, 1536))) return rc;
    int nb = 0;
    if ((rc = stage_regimes(ix, seed_regime, 1, (char *)ix->d_in, nb, st, before != ix->d_in))) return rc;
    const hsa_regime_t *d_reg = (const hsa_regime_t *)ix->d_in;
    const uint8_t *d_bmap = (const uint8_t *)ix->d_in + 256;
    const int seed_max = b->max_len / 3 + 2;
    LaunchPlan P, B, H;
    const bool wide = need_wide(seed_regime, 1);
    if ((rc = plan_launch(ix, (int)calls, seed_max, 0, nb, false, wide, PASS_MAIN, P)) ||
        (rc = plan_launch(ix, (int)calls, seed_max, 0, nb, false, wide, PASS_BIG, B)) ||
        (rc = plan_launch(ix, (int)calls, seed_max, 0, nb, false, wide, PASS_HUGE, H, seed_regime->max_entries)))
        return rc;
    if ((rc = hsa_grow(&ix->d_ovf, &ix->d_ovf_cap, calls * 4 + 64)) ||
        (rc = hsa_grow(&ix->d_ovf2, &ix->d_ovf2_cap, calls * 4 + 64)))
        return rc;
    HSA_HIP(hipMemsetAsync(ctr, 0, 16 * sizeof(unsigned long long), st));
    hipLaunchKernelGGL(k_seed_prep, dim3((unsigned)((2 * n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, S);
    HSA_HIP(hipGetLastError());
    HSA_HIP(hipEventRecord(ix->ev0, st));
    const MgPass mgp{S.mg, S.cw};
    uint32_t *sfl = (uint32_t *)(d + o_fl);
    // qctr 10: the pass's queue head, so that counter [7] (width queries) survives
    if ((rc = launch_pass(ix, P, ix->main, d_reg, d_bmap, S.jobs, S.list, (int)calls, seed_max, 0, S.codes,
                          b->d_n_aln, sfl, b->d_hit_off, b->d_hits, b->hit_cap, ctr, st, (int32_t *)ix->d_ovf, cnt, 10,
                          &mgp)))
        return rc;
    if ((rc = launch_pass(ix, B, ix->big, d_reg, d_bmap, S.jobs, (const int32_t *)ix->d_ovf, (int)calls, seed_max, 0,
                          S.codes, b->d_n_aln, sfl, b->d_hit_off, b->d_hits, b->hit_cap, ctr, st, (int32_t *)ix->d_ovf2,
                          ctr + 8, 9, &mgp, 12)) ||
        (rc = launch_pass(ix, H, ix->huge, d_reg, d_bmap, S.jobs, (const int32_t *)ix->d_ovf2, (int)calls, seed_max, 0,
                          S.codes, b->d_n_aln, sfl, b->d_hit_off, b->d_hits, b->hit_cap, ctr, st, nullptr, ctr + 12, 15,
                          &mgp)))
        return rc;
    HSA_HIP(hipEventRecord(ix->ev1, st));
    return 0;
}

// ---------------------------------------------------------------- splice prefetch
// hsa_splice_prefetch_batch (include/hsa_gpu.h): every width, seed search, anchor search
// and SA -> position lookup bwt_splice_match (bwtgap.c:748-1332) can make before its
// first extension, for a batch of fallback reads, in one device pass.
struct PfArgs {
    RankDir fwd, rev;
    uint32_t T;
    uint32_t C[5];
    uint32_t n, max_len, sc, rs, cws;       // reads, longest, strand-code stride (bytes), row stride, cw stride (pairs)
    const uint32_t *lens;
    const uint64_t *offs;
    const uint8_t *codes;                   // the reads as bwa_seq_t.seq holds them
    const int32_t *amd;                     // per read: the anchors' max_diff
    int32_t seed_max_diff;
    uint8_t *scodes;                        // strand s of read r at (2 r + s) * sc
    int32_t *rows;                          // 6 rows per read, rs pairs each (W1 s0/s1, W12 s0/s1, W0 s0/s1)
    hsa_job_t *jobs;                        // 8 calls per read
    hsa_mg_job_t *mg;
    int32_t *cw;                            // per call cws pairs
    int32_t *list;                          // seed calls, then anchor calls
    int32_t *call_n;                        // 8 n
    uint32_t *call_fl;
    unsigned long long *acount;             // anchor calls listed
    const unsigned long long *d_n;          // the reads' count on the device (hsa_splice_device), or null: n
    uint64_t cwd;                           // the caller-width base is rows: cw starts cwd pairs after it
    uint32_t prefix;                        // seeds read their widths from the W1 rows (HSA_MG_PREFIX)
    const void *ktw;                        // the width trie (hsa_trie.h) for type-1 rows, depth ktd (0: none)
    uint32_t ktd;
};

__device__ __forceinline__ uint32_t pf_n(const PfArgs &a) { return a.d_n ? (uint32_t)*a.d_n : a.n; }

// thread (r, s, kind): kind 0 bwt_cal_width type 1 of the whole strand (and the strand's
// codes), 1 type 1 of its last 12 bases, 2 type 0 of the whole strand (bwtaln.c:73-116;
// the same chains as k_width / k_width0)
__global__ void __launch_bounds__(BLOCK) k_pf_rows(PfArgs a)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t r = t / 6u, s = (t % 6u) & 1u, kind = (t % 6u) >> 1;
    if (r >= pf_n(a)) return;
    const uint32_t L = a.lens[r];
    const uint64_t off = a.offs[r];
    int32_t *const o = a.rows + 2 * ((size_t)r * 6u + kind * 2u + s) * a.rs;
    uint32_t k = 0, l = a.T, bid = 0;
    // the strand's base at p from the 4-byte code word of the last one, held in
    // registers: a chain walks its read one position per step (the codes are 4-byte
    // aligned and padded past the last read)
    uint32_t cq = 0xFFFFFFFFu, cword = 0;
    auto base = [&](uint32_t p) -> uint32_t {
        const uint64_t ix = off + (s ? L - 1u - p : p);
        if ((uint32_t)(ix >> 2) != cq) {
            cword = *reinterpret_cast<const uint32_t *>(a.codes + (ix & ~(uint64_t)3));
            cq = (uint32_t)(ix >> 2);
        }
        const uint32_t c = (cword >> (((uint32_t)ix & 3u) * 8u)) & 0xFFu;
        return s && c < 4 ? 3u - c : c;     // the reverse complement (bwtaln.c:326-333)
    };
    if (kind == 0 || kind == 1) {
        if (kind == 1 && L < 12u) return;
        const uint32_t p0 = kind == 1 ? L - 12u : 0u, n = kind == 1 ? 12u : L;
        uint8_t *const sc = a.scodes + (size_t)(2u * r + s) * a.sc;
        uint32_t tl = 0, tix = 0;            // characters since the last reset and their trie node
        for (uint32_t i = 0; i < n; ++i) {
            const uint32_t c = base(p0 + i);
            if (kind == 0) sc[i] = (uint8_t)c;
            if (c < 4) {
                if (tl < a.ktd) {            // the same forward extension, from the width trie
                    tix = tix * 4u + c;
                    ++tl;
                    trie_w_load<uint32_t>(a.ktw, trie_base(tl) + tix, k, l);
                } else {
                    uint32_t ok, ol;
                    hsa_occ1_pair(a.rev, k, l + 1u, c, ok, ol);
                    const uint32_t cc = hsa_sel4(c, a.C[0], a.C[1], a.C[2], a.C[3]);
                    k = cc + ok + 1u;
                    l = cc + ol;
                }
            }
            if (k > l || c > 3) { k = 0; l = a.T; ++bid; tl = 0; tix = 0; }
            *reinterpret_cast<int2 *>(o + 2 * i) = make_int2((int32_t)(l - k + 1u), (int32_t)bid);
        }
        *reinterpret_cast<int2 *>(o + 2 * n) = make_int2(0, (int32_t)(bid + 1u));
        return;
    }
    *reinterpret_cast<int2 *>(o) = make_int2(0, 0);       // entry 0: never written by the reference
    for (uint32_t i = L - 1u; i > 0 && L > 0; --i) {
        const uint32_t c = base(i);
        if (c < 4) {
            uint32_t ok, ol;
            hsa_occ1_pair(a.fwd, k, l + 1u, c, ok, ol);
            const uint32_t cc = hsa_sel4(c, a.C[0], a.C[1], a.C[2], a.C[3]);
            k = cc + ok + 1u;
            l = cc + ol;
        }
        if (k > l || c > 3) { k = 0; l = a.T; ++bid; }
        *reinterpret_cast<int2 *>(o + 2 * i) = make_int2((int32_t)(l - k + 1u), (int32_t)bid);
    }
    *reinterpret_cast<int2 *>(o + 2 * L) = make_int2(0, (int32_t)(bid + 1u));
}

// thread (r, call 0..5): seed t of strand s (bwtgap.c:797-812): the strand [t sl, t sl + la)
// with width_back = width_seed = the strand prefix's widths (bwt_cal_width of la bases,
// :807): the first la entries of W1 and the terminal {0, bid + 1}
__global__ void __launch_bounds__(BLOCK) k_pf_seeds(PfArgs a)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t r = t / 6u, i = t % 6u, s = i / 3u, tt = i % 3u;
    if (r >= pf_n(a)) return;
    const uint32_t L = a.lens[r], sl = L / 3u, la = sl + (tt == 2u ? L % 3u : 0u);
    const uint32_t call = 8u * r + i;
    a.list[6u * r + i] = (int32_t)call;
    const int32_t *const w1 = a.rows + 2 * ((size_t)r * 6u + s) * a.rs;
    hsa_mg_job_t M;
    if (a.prefix) {                         // the search reads the W1 row's prefix itself
        M.wb_off = ((uint64_t)r * 6u + s) * a.rs;
        M.ws_off = HSA_MG_PREFIX;
    } else {                                // a copy, which the search's width_back export rewrites
        int32_t *const cw = a.cw + 2 * (size_t)call * a.cws;
        for (uint32_t p = 0; p < la; ++p) { cw[2 * p] = w1[2 * p]; cw[2 * p + 1] = w1[2 * p + 1]; }
        cw[2 * la] = 0;
        cw[2 * la + 1] = (la ? w1[2 * (la - 1u) + 1] : 0) + 1;
        M.wb_off = a.cwd + (uint64_t)call * a.cws;
        M.ws_off = 0;
    }
    hsa_job_t J;
    J.off = (uint64_t)(2u * r + s) * a.sc + tt * sl;
    J.len = la;
    J.max_diff = a.seed_max_diff;
    J.seed_len = (int32_t)la;
    J.regime = 0;
    a.jobs[call] = J;
    M.strand = (int32_t)s;
    M.seed = HSA_SEED_ALIAS;
    a.mg[call] = M;
}

// thread (r, s): the 12-mer anchor bwt_splice_match searches after an extension when the
// strand's seed pattern is 3 (seeds 0 and 1 hit: its last 12 bases with their own widths,
// bwtgap.c:911-919) or 6 (seeds 1 and 2: its first 12 with the whole strand's widths,
// :1187-1192); width_seed NULL, the anchor regime, the read's max_diff
__global__ void __launch_bounds__(BLOCK) k_pf_anchors(PfArgs a)
{
    const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t r = t >> 1, s = t & 1u;
    if (r >= pf_n(a)) return;
    const uint32_t L = a.lens[r], call = 8u * r + 6u + s;
    const int32_t *const cn = a.call_n + 8u * r + 3u * s;
    const uint32_t *const cf = a.call_fl + 8u * r + 3u * s;
    const bool done = !(cf[0] & HSA_F_OVERFLOW) && !(cf[1] & HSA_F_OVERFLOW) && !(cf[2] & HSA_F_OVERFLOW);
    const uint32_t mask = (cn[0] > 0) | (cn[1] > 0) << 1 | (cn[2] > 0) << 2;
    if (L <= 12u || !done || (mask != 3u && mask != 6u)) { a.call_n[call] = -1; return; }
    const bool tail = mask == 3u;
    const int32_t *const src = a.rows + 2 * ((size_t)r * 6u + (tail ? 2u : 0u) + s) * a.rs;
    int32_t *const cw = a.cw + 2 * (size_t)call * a.cws;
    for (uint32_t p = 0; p < 13u; ++p) { cw[2 * p] = src[2 * p]; cw[2 * p + 1] = src[2 * p + 1]; }
    hsa_job_t J;
    J.off = (uint64_t)(2u * r + s) * a.sc + (tail ? L - 12u : 0u);
    J.len = 12u;
    J.max_diff = a.amd[r];
    J.seed_len = 0;
    J.regime = 1;
    a.jobs[call] = J;
    hsa_mg_job_t M;
    M.wb_off = a.cwd + (uint64_t)call * a.cws;
    M.ws_off = 0;
    M.strand = (int32_t)s;
    M.seed = HSA_SEED_NONE;
    a.mg[call] = M;
    a.list[6u * a.n + atomicAdd(a.acount, 1ull)] = (int32_t)call;
}

// The SA indices bwt_aln_corelate_check can look up for a call's hits: k .. min(l, k + 49)
// (bwtgap.c:698 reads at most 10 per hit, :711 at most 50; the loop bounds in bwtint_t)
__device__ __forceinline__ uint32_t pf_sa_span(uint32_t k, uint32_t l)
{
    const uint32_t lim = k + 50u;                     // wraps as the reference's bound does
    if (k > l || lim < k) return 0;
    const uint32_t hi = l < lim - 1u ? l : lim - 1u;
    return hi - k + 1u;
}

struct PfSaArgs {
    uint32_t n_calls;
    const int32_t *call_n;
    const uint64_t *call_hit;                // relative to the call's hit region
    const uint32_t *hits_s, *hits_a;         // seed calls' and anchor calls' hit regions
    unsigned long long *call_sa;             // out: first SA result of the call
    unsigned long long *total;
    uint32_t *idx;                           // pass 2: the indices
};

__global__ void __launch_bounds__(BLOCK) k_pf_sa(PfSaArgs a, int fill)
{
    const uint32_t c = blockIdx.x * BLOCK + threadIdx.x;
    if (c >= a.n_calls) return;
    const int32_t n = a.call_n[c];
    if (n <= 0) { if (!fill) a.call_sa[c] = 0; return; }
    const uint32_t *h = ((c & 7u) >= 6u ? a.hits_a : a.hits_s) + a.call_hit[c] * 9u;
    if (!fill) {
        unsigned long long cnt = 0;
        for (int x = 0; x < n; ++x) cnt += pf_sa_span(h[9 * x + 1], h[9 * x + 2]);
        a.call_sa[c] = atomicAdd(a.total, cnt);
        return;
    }
    unsigned long long o = a.call_sa[c];
    for (int x = 0; x < n; ++x) {
        const uint32_t k = h[9 * x + 1], m = pf_sa_span(k, h[9 * x + 2]);
        for (uint32_t j = 0; j < m; ++j) a.idx[o++] = k + j;
    }
}

// The three capacity passes of caller-width searches over a device job list (as
// hsa_splice_seeds_device runs them); counters ctr[16] zeroed here.
static int mg_passes(hsa_index *ix, const hsa_regime_t *d_reg, const uint8_t *d_bmap, int nb, const hsa_job_t *jobs,
                     const int32_t *list, const unsigned long long *n_dev, int n_upper, int max_len, bool gaps, bool wide,
                     int max_entries, const uint8_t *codes, const MgPass &mgp, int32_t *d_n, uint32_t *d_fl,
                     uint64_t *d_ho, uint32_t *d_hits, uint64_t hit_cap, unsigned long long *ctr, hipStream_t st)
{
    int rc;
    LaunchPlan P, B, H;
    if ((rc = plan_launch(ix, n_upper, max_len, 0, nb, gaps, wide, PASS_MAIN, P)) ||
        (rc = plan_launch(ix, n_upper, max_len, 0, nb, gaps, wide, PASS_BIG, B)) ||
        (rc = plan_launch(ix, n_upper, max_len, 0, nb, gaps, wide, PASS_HUGE, H, max_entries)))
        return rc;
    if ((rc = hsa_grow(&ix->d_ovf, &ix->d_ovf_cap, (size_t)n_upper * 4 + 64)) ||
        (rc = hsa_grow(&ix->d_ovf2, &ix->d_ovf2_cap, (size_t)n_upper * 4 + 64)))
        return rc;
    HSA_HIP(hipMemsetAsync(ctr, 0, 16 * sizeof(unsigned long long), st));
    if ((rc = launch_pass(ix, P, ix->main, d_reg, d_bmap, jobs, list, n_upper, max_len, 0, codes, d_n, d_fl, d_ho, d_hits,
                          hit_cap, ctr, st, (int32_t *)ix->d_ovf, n_dev, 10, &mgp)) ||
        (rc = launch_pass(ix, B, ix->big, d_reg, d_bmap, jobs, (const int32_t *)ix->d_ovf, n_upper, max_len, 0, codes, d_n,
                          d_fl, d_ho, d_hits, hit_cap, ctr, st, (int32_t *)ix->d_ovf2, ctr + 8, 9, &mgp, 12)) ||
        (rc = launch_pass(ix, H, ix->huge, d_reg, d_bmap, jobs, (const int32_t *)ix->d_ovf2, n_upper, max_len, 0, codes,
                          d_n, d_fl, d_ho, d_hits, hit_cap, ctr, st, nullptr, ctr + 12, 15, &mgp)))
        return rc;
    return 0;
}

// The prefetch pass, and with ext_rg the splice kernel after it (hsa_splice.hip): res
// receives its per-read answers.
static int pf_batch(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg, int n,
                    const uint32_t *lens, const uint64_t *offs, const uint8_t *codes, size_t codes_len,
                    const int32_t *anchor_max_diff, hsa_splice_pf_t *out, const hsa_regime_t *ext_rg, uint32_t *res,
                    hsa_splice_stats_t *sst)
{
    memset(out, 0, sizeof *out);
    if (sst) memset(sst, 0, sizeof *sst);
    if (n <= 0) return 0;
    if (int rc0 = hsa_need32(ix)) return rc0;
    if (!seed_rg || !anchor_rg || !lens || !offs || !codes || !anchor_max_diff || !out) {
        hsa_set_error("hsa_splice_prefetch_batch: null argument");
        return HSA_E_ARG;
    }
    const hsa_regime_t rg2[2] = {*seed_rg, *anchor_rg};
    int rc = check_regimes(rg2, 2);
    if (rc) return rc;
    if (seed_rg->max_gapo != 0) { hsa_set_error("seed searches have no gap opens (bwtgap.c:772)"); return HSA_E_ARG; }
    if (!fast_regimes(rg2, 2)) { hsa_set_error("splice prefetch: options outside k_search's layouts"); return HSA_E_ARG; }
    uint32_t M = 0;
    for (int r = 0; r < n; ++r) {
        if (lens[r] < 3 || lens[r] > 3 * (FAST_MAX_LEN - 2)) {    // seeds of at most FAST_MAX_LEN bases
            hsa_set_error("splice prefetch: read %d of %u bases", r, lens[r]);
            return HSA_E_ARG;
        }
        if (offs[r] > codes_len || lens[r] > codes_len - offs[r]) { hsa_set_error("read %d past codes_len", r); return HSA_E_ARG; }
        if (anchor_max_diff[r] > anchor_rg->max_diff) { hsa_set_error("read %d: max_diff above the regime's", r); return HSA_E_ARG; }
        M = lens[r] > M ? lens[r] : M;
    }
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = ix->stream;
    const double t0 = [] { struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t); return t.tv_sec + 1e-9 * t.tv_nsec; }();
    const size_t N = (size_t)n, calls = 8 * N;
    const uint32_t sc = (M + 15u) / 16u * 16u + 16u, rs = M + 1u, cws = M / 3u + 3u > 13u ? M / 3u + 3u : 13u;
    const uint64_t cap_s = 6 * N * 16 + 65536, cap_a = 2 * N * 16 + 16384;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    // device layout
    size_t o = 0;
    const size_t o_lens = o; o += al(N * 4);
    const size_t o_offs = o; o += al(N * 8);
    const size_t o_amd = o; o += al(N * 4);
    const size_t o_codes = o; o += al(codes_len + 64);
    const size_t o_sc = o; o += al(2 * N * sc + 64);
    const size_t o_jobs = o; o += al(calls * sizeof(hsa_job_t));
    const size_t o_mg = o; o += al(calls * sizeof(hsa_mg_job_t));
    const size_t o_list = o; o += al(8 * N * 4);
    const size_t o_ctr = o; o += 1024;                    // seed ctr[16], anchor ctr[16], anchor count, SA total
    // outputs, one contiguous block: [call_n | call_fl | call_hit | call_sa | rows | cw | hits_s | hits_a]
    const size_t o_out = o;
    const size_t q_n = 0, q_fl = q_n + al(calls * 4), q_ho = q_fl + al(calls * 4), q_sa = q_ho + al(calls * 8);
    const size_t q_rows = q_sa + al(calls * 8), q_cw = q_rows + al(N * 6 * rs * 8), q_hs = q_cw + al(calls * cws * 8);
    const size_t q_ha = q_hs + al(cap_s * 36), q_end = q_ha + al(cap_a * 36);
    o += q_end;
    const size_t o_res = o; o += ext_rg ? al(N * HSA_SP_RES_WORDS * 4) : 0;   // the splice kernel's answers
    if ((rc = hsa_grow(&ix->d_pf, &ix->d_pf_cap, o + 256))) return rc;
    char *d = (char *)ix->d_pf;
    HSA_HIP(hipMemcpyAsync(d + o_lens, lens, N * 4, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(d + o_offs, offs, N * 8, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(d + o_amd, anchor_max_diff, N * 4, hipMemcpyHostToDevice, st));
    HSA_HIP(hipMemcpyAsync(d + o_codes, codes, codes_len, hipMemcpyHostToDevice, st));
    unsigned long long *ctr_s = (unsigned long long *)(d + o_ctr), *ctr_a = ctr_s + 16, *acnt = ctr_s + 32,
                       *satot = ctr_s + 33, *scnt = ctr_s + 34;
    HSA_HIP(hipMemsetAsync(ctr_s, 0, 1024, st));
    char *dq = d + o_out;
    PfArgs A;
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.T = ix->T;
    memcpy(A.C, ix->C, sizeof A.C);
    A.n = (uint32_t)n; A.max_len = M; A.sc = sc; A.rs = rs; A.cws = cws;
    A.lens = (const uint32_t *)(d + o_lens); A.offs = (const uint64_t *)(d + o_offs);
    A.codes = (const uint8_t *)(d + o_codes); A.amd = (const int32_t *)(d + o_amd);
    A.seed_max_diff = seed_rg->max_diff;
    A.scodes = (uint8_t *)(d + o_sc);
    A.rows = (int32_t *)(dq + q_rows);
    A.jobs = (hsa_job_t *)(d + o_jobs); A.mg = (hsa_mg_job_t *)(d + o_mg);
    A.cw = (int32_t *)(dq + q_cw); A.list = (int32_t *)(d + o_list);
    A.call_n = (int32_t *)(dq + q_n); A.call_fl = (uint32_t *)(dq + q_fl);
    A.acount = acnt;
    A.d_n = nullptr;
    A.cwd = (q_cw - q_rows) / 8;
    {
        const char *te = getenv("HSA_TRIE");
        const bool tr = ix->trie_depth > 0 && !ix->trie_wide && !(te && atoi(te) == 0);
        A.ktw = tr ? ix->d_trie_w : nullptr;
        A.ktd = tr ? ix->trie_depth : 0u;
    }
    A.prefix = ext_rg ? 1u : 0u;             // the host tables want every call's width_back after it
    HSA_HIP(hipMemsetAsync(d + o_sc, 4, 2 * N * sc + 64, st));         // padding reads as N
    hipLaunchKernelGGL(k_pf_rows, dim3((unsigned)((6 * N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, A);
    hipLaunchKernelGGL(k_pf_seeds, dim3((unsigned)((6 * N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, A);
    HSA_HIP(hipGetLastError());
    // both regimes staged once: seeds use regime 0, anchors regime 1
    void *before = ix->d_in;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, 1536))) return rc;
    int nb = 0;
    if ((rc = stage_regimes(ix, rg2, 2, (char *)ix->d_in, nb, st, before != ix->d_in))) return rc;
    const hsa_regime_t *d_reg = (const hsa_regime_t *)ix->d_in;
    const uint8_t *d_bmap = (const uint8_t *)ix->d_in + 256;
    const bool wide = need_wide(rg2, 2);
    const MgPass mgp{A.mg, A.rows};          // widths at rows + wb_off (a row's prefix, or cw + call * cws)
    const unsigned long long n_seed = 6 * N;
    HSA_HIP(hipMemcpyAsync(scnt, &n_seed, 8, hipMemcpyHostToDevice, st));
    HSA_HIP(hipEventRecord(ix->ev0, st));
    if ((rc = mg_passes(ix, d_reg, d_bmap, nb, A.jobs, A.list, scnt, (int)(6 * N), (int)(M / 3u + 2u), false, wide,
                        seed_rg->max_entries, A.scodes, mgp, A.call_n, A.call_fl, (uint64_t *)(dq + q_ho),
                        (uint32_t *)(dq + q_hs), cap_s, ctr_s, st)))
        return rc;
    hipLaunchKernelGGL(k_pf_anchors, dim3((unsigned)((2 * N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, A);
    HSA_HIP(hipGetLastError());
    // the anchors' pass is planned for the anchors there are (a gapped regime's pool per
    // lane is large: planning for all 2 n strands would size the scratch for them)
    unsigned long long n_anchor = 0;
    HSA_HIP(hipMemcpyAsync(&n_anchor, acnt, 8, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    if (n_anchor &&
        (rc = mg_passes(ix, d_reg, d_bmap, nb, A.jobs, A.list + 6 * N, acnt, (int)n_anchor, 12,
                        anchor_rg->max_gapo > 0, wide, anchor_rg->max_entries, A.scodes, mgp, A.call_n, A.call_fl,
                        (uint64_t *)(dq + q_ho), (uint32_t *)(dq + q_ha), cap_a, ctr_a, st)))
        return rc;
    // unfinished calls (hits past the caps, stacks past the HUGE pass) are not answered
    PfSaArgs S;
    S.n_calls = (uint32_t)calls;
    S.call_n = A.call_n; S.call_hit = (const uint64_t *)(dq + q_ho);
    S.hits_s = (const uint32_t *)(dq + q_hs); S.hits_a = (const uint32_t *)(dq + q_ha);
    S.call_sa = (unsigned long long *)(dq + q_sa); S.total = satot; S.idx = nullptr;
    if (ext_rg) {
        // bwt_splice_match itself (hsa_splice.hip); the host tables (SA lookups, the pinned
        // copy) serve only the host's bwt_splice_match, which the caller runs with its own
        // prefetch for the reads the kernel hands back
        HSA_HIP(hipEventRecord(ix->ev1, st));
        PfDev pd;
        pd.n = (uint32_t)n; pd.max_len = M; pd.sc = sc; pd.rs = rs; pd.cws = cws;
        pd.lens = A.lens; pd.amd = A.amd; pd.scodes = A.scodes; pd.rows = A.rows; pd.cw = A.cw;
        pd.call_n = A.call_n; pd.call_fl = A.call_fl; pd.call_hit = (const uint64_t *)(dq + q_ho);
        pd.hits_s = (const uint32_t *)(dq + q_hs); pd.hits_a = (const uint32_t *)(dq + q_ha);
        pd.d_n = nullptr; pd.idx = nullptr;
        if ((rc = hsa_splice_device_launch(ix, pd, *ext_rg, (uint32_t *)(d + o_res), ctr_s + 40, st))) return rc;
        HSA_HIP(hipEventRecord(ix->ev_sp, st));
        HSA_HIP(hipMemcpyAsync(res, d + o_res, N * HSA_SP_RES_WORDS * 4, hipMemcpyDeviceToHost, st));
        unsigned long long sc4[4];
        HSA_HIP(hipMemcpyAsync(sc4, ctr_s + 40, sizeof sc4, hipMemcpyDeviceToHost, st));
        HSA_HIP(hipStreamSynchronize(st));
        float ms = 0, sms = 0;
        HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
        HSA_HIP(hipEventElapsedTime(&sms, ix->ev1, ix->ev_sp));
        out->n = n; out->max_len = (int)M; out->row_stride = (int)rs; out->cw_stride = (int)cws;
        out->kernel_ms = ms;
        if (sst) {
            sst->kernel_ms = sms;
            sst->extensions = sc4[0]; sst->pops = sc4[1]; sst->sa_lookups = sc4[2]; sst->not_answered = sc4[3];
        }
        return 0;
    }
    const bool with_sa = ix->d_sa != nullptr;
    if (with_sa) hipLaunchKernelGGL(k_pf_sa, dim3((unsigned)((calls + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, S, 0);
    HSA_HIP(hipGetLastError());
    unsigned long long hc[40];
    HSA_HIP(hipMemcpyAsync(hc, ctr_s, sizeof hc, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    const uint64_t n_sa = with_sa ? hc[33] : 0;
    if (n_sa && (rc = hsa_grow(&ix->d_pf2, &ix->d_pf2_cap, al(n_sa * 4) + n_sa * 16 + 256))) return rc;
    uint32_t *d_idx = (uint32_t *)ix->d_pf2, *d_sao = (uint32_t *)((char *)ix->d_pf2 + al(n_sa * 4));
    if (n_sa) {
        S.idx = d_idx;
        hipLaunchKernelGGL(k_pf_sa, dim3((unsigned)((calls + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, S, 1);
        HSA_HIP(hipGetLastError());
        if ((rc = hsa_sa_position_device(ix, n_sa, d_idx, d_sao, st))) return rc;
    }
    HSA_HIP(hipEventRecord(ix->ev1, st));
    // one copy of the output block (hits up to their counts) into pinned host memory
    const uint64_t nh_s = hc[1] < cap_s ? hc[1] : cap_s, nh_a = hc[16 + 1] < cap_a ? hc[16 + 1] : cap_a;
    const size_t h_need = q_hs + (nh_s + nh_a) * 36 + al(n_sa * 16) + 256;
    if (h_need > ix->h_pf_cap) {
        if (ix->h_pf) (void)hipHostFree(ix->h_pf);
        ix->h_pf = nullptr; ix->h_pf_cap = 0;
        const size_t want = h_need + h_need / 4 > ((size_t)64 << 20) ? h_need + h_need / 4 : ((size_t)64 << 20);
        HSA_HIP(hipHostMalloc(&ix->h_pf, want, hipHostMallocDefault));
        ix->h_pf_cap = want;
    }
    char *h = (char *)ix->h_pf;
    HSA_HIP(hipMemcpyAsync(h, dq, q_hs + nh_s * 36, hipMemcpyDeviceToHost, st));
    if (nh_a) HSA_HIP(hipMemcpyAsync(h + q_hs + nh_s * 36, dq + q_ha, nh_a * 36, hipMemcpyDeviceToHost, st));
    const size_t h_sa = al(q_hs + (nh_s + nh_a) * 36);
    if (n_sa) HSA_HIP(hipMemcpyAsync(h + h_sa, d_sao, n_sa * 16, hipMemcpyDeviceToHost, st));
    HSA_HIP(hipStreamSynchronize(st));
    float ms = 0;
    HSA_HIP(hipEventElapsedTime(&ms, ix->ev0, ix->ev1));
    // anchor calls' hit offsets into the one hits array; unfinished calls -2
    int32_t *cn = (int32_t *)(h + q_n);
    const uint32_t *cf = (const uint32_t *)(h + q_fl);
    uint64_t *ch = (uint64_t *)(h + q_ho);
    for (size_t c = 0; c < calls; ++c) {
        if ((c & 7u) >= 6u && cn[c] >= 0) ch[c] += nh_s;
        if (cn[c] >= 0 && (cf[c] & HSA_F_OVERFLOW)) cn[c] = -2;
    }
    out->n = n; out->max_len = (int)M; out->row_stride = (int)rs; out->cw_stride = (int)cws;
    out->call_n = cn; out->call_hit = ch;
    out->call_sa = with_sa ? (const uint64_t *)(h + q_sa) : nullptr;
    out->rows = (const int32_t *)(h + q_rows);
    out->wafter = (const int32_t *)(h + q_cw);
    out->hits = (const uint32_t *)(h + q_hs);
    out->sa = n_sa ? (const uint32_t *)(h + h_sa) : nullptr;
    out->n_hits = nh_s + nh_a; out->n_sa = n_sa;
    out->kernel_ms = ms;
    if (getenv("HSA_VERBOSE")) {
        struct timespec t; clock_gettime(CLOCK_MONOTONIC, &t);
        fprintf(stderr, "[hsa] splice prefetch on the device: %d reads, %llu seed + %llu anchor calls, %llu hits, %llu SA "
                        "lookups, %.1f ms (kernels %.1f ms)\n", n, (unsigned long long)n_seed, (unsigned long long)hc[32],
                (unsigned long long)(nh_s + nh_a), (unsigned long long)n_sa, 1e3 * (t.tv_sec + 1e-9 * t.tv_nsec - t0), ms);
    }
    return 0;
}

// ---------------------------------------------------------------- hsa_splice_device
// The fallback reads of a device batch (the main pass flagged them), compacted: their
// order does not matter, a read's splice path depends on the read alone.  A job whose
// length is outside [3, max_len] (the prefetch's rows and codes are sized from max_len)
// is not taken: its answer is HSA_SP_WIN (not answered), so a caller runs the host's
// path for it.
__global__ void __launch_bounds__(BLOCK) k_sp_prep(const hsa_job_t *jobs, const uint32_t *flags, const int32_t *n_aln,
                                                   uint32_t n, uint32_t max_len, uint32_t *res, uint32_t *lens,
                                                   uint64_t *offs, int32_t *amd, int32_t *idx, unsigned long long *cnt)
{
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= n || !(flags[j] & HSA_F_FALLBACK) || n_aln[j] != 0) return;
    const hsa_job_t J = jobs[j];
    if (J.len < 3u || J.len > max_len) {
        res[(size_t)j * HSA_SP_RES_WORDS] = HSA_SP_WIN;
        res[(size_t)j * HSA_SP_RES_WORDS + 1] = 0u;
        return;
    }
    const uint32_t r = (uint32_t)atomicAdd(cnt, 1ull);
    lens[r] = J.len;
    offs[r] = J.off;
    amd[r] = J.max_diff;
    idx[r] = (int32_t)j;
}

__global__ void k_sp_calls(const unsigned long long *cnt, unsigned long long *scnt) { *scnt = 6ull * *cnt; }

// the batch's counters: [0] reads, [5] rank queries of the seed and anchor searches and
// their widths, [6] their hits ([1]-[4] come from the splice kernel)
__global__ void k_sp_stats(const unsigned long long *cnt, const unsigned long long *ctr_s,
                           const unsigned long long *ctr_a, unsigned long long *out)
{
    out[0] = *cnt;
    out[5] = ctr_s[2] + ctr_s[7] + ctr_a[2] + ctr_a[7];
    out[6] = ctr_s[1] + ctr_a[1];
}

extern "C" int hsa_splice_device(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg,
                                 const hsa_regime_t *ext_rg, const hsa_splice_batch_t *b, void *stream)
{
    if (int rc0 = hsa_need32(ix)) return rc0;
    if (!seed_rg || !anchor_rg || !ext_rg || !b) { hsa_set_error("hsa_splice_device: null argument"); return HSA_E_ARG; }
    const hsa_regime_t rg2[2] = {*seed_rg, *anchor_rg};
    int rc = check_regimes(rg2, 2);
    if (rc) return rc;
    if (seed_rg->max_gapo != 0) { hsa_set_error("seed searches have no gap opens (bwtgap.c:772)"); return HSA_E_ARG; }
    if (!fast_regimes(rg2, 2)) { hsa_set_error("splice path: options outside k_search's layouts"); return HSA_E_ARG; }
    if (b->max_len < 3 || b->max_len > 3 * (FAST_MAX_LEN - 2) || b->n_jobs < 0) {
        hsa_set_error("hsa_splice_device: max_len %d / n_jobs %d out of range", b->max_len, b->n_jobs);
        return HSA_E_ARG;
    }
    if (b->n_jobs == 0) return 0;
    HSA_HIP(hipSetDevice(ix->device));
    hipStream_t st = stream ? (hipStream_t)stream : ix->stream;
    const size_t N = (size_t)b->n_jobs, calls = 8 * N;
    const uint32_t M = (uint32_t)b->max_len;
    const uint32_t sc = (M + 15u) / 16u * 16u + 16u, rs = M + 1u, cws = M / 3u + 3u > 13u ? M / 3u + 3u : 13u;
    const uint64_t cap_s = 6 * N * 16 + 65536, cap_a = 2 * N * 16 + 16384;
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    size_t o = 0;
    const size_t o_lens = o; o += al(N * 4);
    const size_t o_offs = o; o += al(N * 8);
    const size_t o_amd = o; o += al(N * 4);
    const size_t o_idx = o; o += al(N * 4);
    const size_t o_sc = o; o += al(2 * N * sc + 64);
    const size_t o_jobs = o; o += al(calls * sizeof(hsa_job_t));
    const size_t o_mg = o; o += al(calls * sizeof(hsa_mg_job_t));
    const size_t o_list = o; o += al(8 * N * 4);
    const size_t o_ctr = o; o += 1024;
    const size_t o_n = o; o += al(calls * 4);
    const size_t o_fl = o; o += al(calls * 4);
    const size_t o_ho = o; o += al(calls * 8);
    const size_t o_rows = o; o += al(N * 6 * rs * 8);
    const size_t o_cw = o; o += al(calls * cws * 8);
    const size_t o_hs = o; o += al(cap_s * 36);
    const size_t o_ha = o; o += al(cap_a * 36);
    if ((rc = hsa_grow(&ix->d_pf, &ix->d_pf_cap, o + 256))) return rc;
    char *d = (char *)ix->d_pf;
    unsigned long long *ctr_s = (unsigned long long *)(d + o_ctr), *ctr_a = ctr_s + 16, *acnt = ctr_s + 32,
                       *scnt = ctr_s + 34, *rcnt = ctr_s + 35;
    unsigned long long *out_ctr = (unsigned long long *)b->d_counters;
    HSA_HIP(hipMemsetAsync(ctr_s, 0, 1024, st));
    HSA_HIP(hipMemsetAsync(out_ctr, 0, 8 * sizeof(unsigned long long), st));
    PfArgs A;
    A.fwd = RankDir{ix->blk[0], ix->isa0};
    A.rev = RankDir{ix->blk[1], ix->risa0};
    A.T = ix->T;
    memcpy(A.C, ix->C, sizeof A.C);
    A.n = (uint32_t)N; A.max_len = M; A.sc = sc; A.rs = rs; A.cws = cws;
    A.lens = (const uint32_t *)(d + o_lens); A.offs = (const uint64_t *)(d + o_offs);
    A.codes = b->d_codes; A.amd = (const int32_t *)(d + o_amd);
    A.seed_max_diff = seed_rg->max_diff;
    A.scodes = (uint8_t *)(d + o_sc);
    A.rows = (int32_t *)(d + o_rows);
    A.jobs = (hsa_job_t *)(d + o_jobs); A.mg = (hsa_mg_job_t *)(d + o_mg);
    A.cw = (int32_t *)(d + o_cw); A.list = (int32_t *)(d + o_list);
    A.call_n = (int32_t *)(d + o_n); A.call_fl = (uint32_t *)(d + o_fl);
    A.acount = acnt;
    A.d_n = rcnt;
    A.cwd = (o_cw - o_rows) / 8;
    {
        const char *te = getenv("HSA_TRIE");
        const bool tr = ix->trie_depth > 0 && !ix->trie_wide && !(te && atoi(te) == 0);
        A.ktw = tr ? ix->d_trie_w : nullptr;
        A.ktd = tr ? ix->trie_depth : 0u;
    }
    A.prefix = 1;
    const unsigned grid_n = (unsigned)((N + BLOCK - 1) / BLOCK);
    hipLaunchKernelGGL(k_sp_prep, dim3(grid_n), dim3(BLOCK), 0, st, b->d_jobs, b->d_flags, b->d_n_aln, (uint32_t)N,
                       M, b->d_res, (uint32_t *)(d + o_lens), (uint64_t *)(d + o_offs), (int32_t *)(d + o_amd), (int32_t *)(d + o_idx),
                       rcnt);
    hipLaunchKernelGGL(k_sp_calls, dim3(1), dim3(1), 0, st, (const unsigned long long *)rcnt, scnt);
    HSA_HIP(hipMemsetAsync(d + o_sc, 4, 2 * N * sc + 64, st));         // padding reads as N
    hipLaunchKernelGGL(k_pf_rows, dim3((unsigned)((6 * N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, A);
    hipLaunchKernelGGL(k_pf_seeds, dim3((unsigned)((6 * N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, A);
    HSA_HIP(hipGetLastError());
    void *before = ix->d_in;
    if ((rc = hsa_grow(&ix->d_in, &ix->d_in_cap, 1536))) return rc;
    int nb = 0;
    if ((rc = stage_regimes(ix, rg2, 2, (char *)ix->d_in, nb, st, before != ix->d_in))) return rc;
    const hsa_regime_t *d_reg = (const hsa_regime_t *)ix->d_in;
    const uint8_t *d_bmap = (const uint8_t *)ix->d_in + 256;
    const bool wide = need_wide(rg2, 2);
    const MgPass mgp{A.mg, A.rows};          // widths at rows + wb_off (a row's prefix, or cw + call * cws)
    // no host round trip: the passes take their job counts from the device (the seed
    // calls' 6 per read, the anchors k_pf_anchors listed), planned for their upper bounds
    if ((rc = mg_passes(ix, d_reg, d_bmap, nb, A.jobs, A.list, scnt, (int)(6 * N), (int)(M / 3u + 2u), false, wide,
                        seed_rg->max_entries, A.scodes, mgp, A.call_n, A.call_fl, (uint64_t *)(d + o_ho),
                        (uint32_t *)(d + o_hs), cap_s, ctr_s, st)))
        return rc;
    hipLaunchKernelGGL(k_pf_anchors, dim3((unsigned)((2 * N + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, st, A);
    HSA_HIP(hipGetLastError());
    if ((rc = mg_passes(ix, d_reg, d_bmap, nb, A.jobs, A.list + 6 * N, acnt, (int)(2 * N), 12, anchor_rg->max_gapo > 0,
                        wide, anchor_rg->max_entries, A.scodes, mgp, A.call_n, A.call_fl, (uint64_t *)(d + o_ho),
                        (uint32_t *)(d + o_ha), cap_a, ctr_a, st)))
        return rc;
    PfDev pd;
    pd.n = (uint32_t)N; pd.max_len = M; pd.sc = sc; pd.rs = rs; pd.cws = cws;
    pd.lens = A.lens; pd.amd = A.amd; pd.scodes = A.scodes; pd.rows = A.rows; pd.cw = A.cw;
    pd.call_n = A.call_n; pd.call_fl = A.call_fl; pd.call_hit = (const uint64_t *)(d + o_ho);
    pd.hits_s = (const uint32_t *)(d + o_hs); pd.hits_a = (const uint32_t *)(d + o_ha);
    pd.d_n = rcnt; pd.idx = (const int32_t *)(d + o_idx);
    if ((rc = hsa_splice_device_launch(ix, pd, *ext_rg, b->d_res, out_ctr + 1, st))) return rc;
    hipLaunchKernelGGL(k_sp_stats, dim3(1), dim3(1), 0, st, (const unsigned long long *)rcnt,
                       (const unsigned long long *)ctr_s, (const unsigned long long *)ctr_a, out_ctr);
    HSA_HIP(hipGetLastError());
    return 0;
}

extern "C" int hsa_splice_prefetch_batch(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg,
                                         int n, const uint32_t *lens, const uint64_t *offs, const uint8_t *codes,
                                         size_t codes_len, const int32_t *anchor_max_diff, hsa_splice_pf_t *out)
{
    return pf_batch(ix, seed_rg, anchor_rg, n, lens, offs, codes, codes_len, anchor_max_diff, out, nullptr, nullptr,
                    nullptr);
}

extern "C" int hsa_splice_match_batch(hsa_index_t *ix, const hsa_regime_t *seed_rg, const hsa_regime_t *anchor_rg,
                                      const hsa_regime_t *ext_rg, int n, const uint32_t *lens, const uint64_t *offs,
                                      const uint8_t *codes, size_t codes_len, const int32_t *anchor_max_diff,
                                      hsa_splice_pf_t *pf, uint32_t *res, hsa_splice_stats_t *stats)
{
    if (!ext_rg || (n > 0 && !res) || !pf) {
        hsa_set_error("hsa_splice_match_batch: null argument");
        return HSA_E_ARG;
    }
    return pf_batch(ix, seed_rg, anchor_rg, n, lens, offs, codes, codes_len, anchor_max_diff, pf, ext_rg, res, stats);
}

extern "C" int hsa_pass_times(hsa_index_t *ix, int n, float *widths_ms, float *search_ms)
{
    if (n < 1 || n > hsa_index::PASS_RING || (uint64_t)n > ix->pev_n) {
        hsa_set_error("hsa_pass_times: %d passes requested, %llu recorded (ring %d)", n,
                      (unsigned long long)ix->pev_n, hsa_index::PASS_RING);
        return HSA_E_ARG;
    }
    for (int i = 0; i < n; ++i) {
        hipEvent_t *pe = ix->pev[(ix->pev_n - (uint64_t)n + (uint64_t)i) % hsa_index::PASS_RING];
        HSA_HIP(hipEventSynchronize(pe[2]));
        HSA_HIP(hipEventElapsedTime(widths_ms + i, pe[0], pe[1]));
        HSA_HIP(hipEventElapsedTime(search_ms + i, pe[1], pe[2]));
    }
    return 0;
}

extern "C" int hsa_last_pass_ms(hsa_index_t *ix, float *widths_ms, float *search_ms)
{
    if (ix->pev_n) return hsa_pass_times(ix, 1, widths_ms, search_ms);   // the newest hsa_search_device pass
    HSA_HIP(hipEventSynchronize(ix->ev1));
    HSA_HIP(hipEventElapsedTime(widths_ms, ix->ev0, ix->evm));
    HSA_HIP(hipEventElapsedTime(search_ms, ix->evm, ix->ev1));
    return 0;
}
