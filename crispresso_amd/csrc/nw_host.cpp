// nw_host.cpp -- C ABI (include/crispr_nw.h) over the gfx950 alignment kernel.
//
// Owns one HIP stream and the device buffers of one GPU.  Everything the
// reference did by spawning `needle` (CRISPRessoCORE.py:1788-1936) happens here
// in-process: the amplicon becomes a substitution profile in HBM, reads are
// copied once, one kernel aligns the whole batch, results come back as the
// three alignment strings plus per-read statistics.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cctype>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/crispr_nw.h"
#include "host_pool.h"
#include "nw_device.h"
#include "nw_edna.h"

namespace {

constexpr int kMaxRef = 8192;       // the exact multi-wave kernel (nw_exact.hip)
constexpr int kMaxRefWave = 1024;   // the band, stream and one-wave kernels
constexpr int kMaxLds = 160 * 1024;

template <class T>
struct DevBuf {
    T* p = nullptr;
    size_t cap = 0;  // elements
    hipError_t reserve(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc((void**)&p, std::max<size_t>(n, 1) * sizeof(T));
        if (e == hipSuccess) cap = n;
        return e;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

// One amplicon's device tables (pointers into nw_ctx::d_arena).
struct Profile {
    const int8_t* prof = nullptr;      // [NCODE][64][RP] int8: exact kernel
    const uint32_t* rowpos = nullptr;  // band walk: codes each row scores > 0 against
    const uint8_t* amp = nullptr;      // amplicon bytes (+16 pad)
    int R = 0;
    // window seeds (classify, packed input): the amplicon 2 bits per base (the reads' packing) and
    // its A C G T 16-mers sorted by (key, position); null for amplicons over 1024 bp
    const uint32_t* amp2 = nullptr;
    const uint32_t* seed_key = nullptr;
    const uint16_t* seed_pos = nullptr;
    int32_t n_seed = 0;
    // classify's LDS image of the amplicon (cls_image): copied as it is by every block
    const uint32_t* cls_img = nullptr;
    int32_t cls_words = 0;
    bool amp_acgt = false;             // every amplicon byte A C G T (either case)
};

// Device buffers of one chunk's kernels.  The pipelined calls alternate two sets on
// two compute streams, so a chunk's latency-bound tail (second band level, exact
// kernel, compaction) overlaps the next chunk's bulk kernels.
struct Scratch {
    DevBuf<uint8_t> d_tb;              // exact kernel: traceback slabs when they do not fit LDS
    DevBuf<int64_t> d_fallback;        // reads the 16 / 32-diagonal levels gave up on (the wide level's input)
    DevBuf<int32_t> d_seed;            // seeded band: per read of the chunk, its hits' diagonals (seed_pack)
    DevBuf<int32_t> d_seed2;           // ... and its blocks' facts for the refined certificate (seed2_pack)
    DevBuf<int32_t> d_seed_list;       // seeded band: the chunk's seeded reads (the segment sort's third list)
    DevBuf<uint8_t> d_seed_flags;      // ... per entry: left to the wide level by the 32-diagonal level
    DevBuf<int32_t> d_seed_list2;      // ... those entries, in order (the wide level's seeded list)
    DevBuf<int64_t> d_fallback2;       // reads the wide level gave up on (the exact kernel's list)
    DevBuf<int32_t> d_fallback_count;  // [0] fallback count, [1] -, [2] redo count
    DevBuf<int32_t> d_redo;            // reads the first band level could not certify
    DevBuf<uint8_t> d_redo_flags;      // per sorted position: handed to the second level
    DevBuf<int32_t> d_order, d_sort_key;
    DevBuf<int32_t> d_cert_q, d_cert_cnt;   // classify's queues for nw_band_cert (KernelArgs::cert_q)
    DevBuf<unsigned long long> d_lb;   // look-back words of the single-pass scans (sort, redo list, ops)
    DevBuf<uint8_t> d_bregion;         // band regions (per read pair)
    DevBuf<uint32_t> d_slots, d_spill, d_staging;   // ops output: run slots, spill area, compaction output
    DevBuf<int32_t> d_nops, d_opsctl;
    void release() {
        d_tb.release(); d_fallback.release(); d_fallback2.release(); d_fallback_count.release(); d_redo.release();
        d_redo_flags.release(); d_order.release(); d_sort_key.release(); d_lb.release();
        d_cert_q.release(); d_cert_cnt.release();
        d_seed.release(); d_seed2.release(); d_seed_list.release(); d_seed_flags.release(); d_seed_list2.release();
        d_bregion.release(); d_slots.release(); d_spill.release(); d_staging.release(); d_nops.release();
        d_opsctl.release();
    }
};
constexpr int kScratchSets = 6;   // 3 per pass of a dual call, 3 otherwise
constexpr int kComputeStreams = 3;
constexpr int64_t kWidePairs = 2048;     // read pairs of one chunk's wide level (region capacity)

// Test switches (environment, read per call).  Each forces a path the defaults reach only on
// particular inputs, so the tests can hold every path to the oracle:
//   CRISPR_NW_KERNEL     "full": every read through the exact int32 kernel; "diag32": the band
//                        path without its 16-diagonal level
//   CRISPR_NW_EXACT      "multi[:grid]": the exact work lists through the multi-wave kernel (the
//                        first `grid` entries, the rest through the one-wave kernel); "lds": the
//                        one-wave kernel keeps its traceback in LDS however few waves fit
//   CRISPR_NW_WIDE       "0": no 128-diagonal level
//   CRISPR_NW_DIRECT     reads up to which a chunk's first level hands straight to the wide level
//   CRISPR_NW_L1SKIP     "0": chunks of >= 65536 reads with few DP reads keep the first level
//   CRISPR_NW_ADAPT      "0": no adaptive level choice across chunks
//   CRISPR_NW_CHUNK, CRISPR_NW_OPS_SLOT, CRISPR_NW_SPILL_WORDS, CRISPR_NW_REGION_MB: sizes
//                        (chunk reads, runs per slot, spill words, band region MB)
// and CRISPR_NW_HOST_TIMING=1 (diagnostics: the host's phase split of a call on stderr).

struct nw_ctx {
    int device = 0;
    int num_cus = 256;
    hipStream_t stream = nullptr;
    Scratch sc[kScratchSets];
    Scratch* s = &sc[0];                               // the set launch_range / configure use
    hipStream_t cs = nullptr;                          // the stream launch_range queues on
    hipStream_t cstream[kComputeStreams] = {};            // compute stream of each set ([0] = stream)
    // tail split (ops_call): launch_range queues a chunk's first band level on
    // c->cs, then records split_ev there and moves to split_to for the rest (second level,
    // exact kernel, compaction)
    hipStream_t split_to = nullptr;
    hipEvent_t split_ev = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev_fill = nullptr, ev_walk = nullptr;   // after the fill / walk kernels
    hipEvent_t ev_sort = nullptr, ev_l2 = nullptr;     // band path: after the sort, after the second level
    bool phases = false;                               // record the phase events (nw_batch_run_async)
    std::string err;
    // params
    float gap_open_f = 10.0f, gap_extend_f = 0.5f;
    int scale = 2, gap_open = 20, gap_extend = 1;
    bool end_weight = false;           // needle -endweight: end gaps cost end_open + (k-1) end_extend
    int end_open = 20, end_extend = 1; // scaled
    // reference
    std::string ref;
    DevBuf<uint8_t> d_arena;          // every amplicon's tables (upload_profiles)
    // what d_arena / the shared tables hold (a repeated pooled call reuses them)
    std::vector<std::string> arena_refs;
    std::vector<Profile> arena_profs;
    std::string arena_key, shared_key;
    Profile cur{};                    // the amplicon being aligned
    DevBuf<uint8_t> d_lut6, d_lut;
    // batch
    int64_t n = 0;
    int32_t lb_max = 0;
    int64_t stride = 0;
    int64_t cells = 0;
    std::vector<int32_t> read_lens;
    DevBuf<uint8_t> d_reads;
    DevBuf<uint8_t> d_packed, d_exc_byte;   // 2-bit packed input (nw_align_ops_packed) and its exceptions
    DevBuf<int64_t> d_exc_pos;
    DevBuf<int64_t> d_offsets;
    // packed calls: the chunks' length segments (nw::LenSeg), pinned on the host and in HBM
    DevBuf<uint8_t> d_lens;
    uint8_t* h_lens = nullptr;
    int64_t h_lens_cap = 0;
    DevBuf<uint8_t> d_out;
    DevBuf<nw::Stat> d_stats;
    nw::LaunchCfg cfg{};              // full-storage kernel
    // certified diagonal-band kernels (nw_band.hip): the default path
    bool use_diag = false;
    nw::LaunchCfg diag_fill{}, diag_walk{};          // 32-diagonal level (the certificate's last resort)
    nw::LaunchCfg diag16_fill{}, diag16_walk{};      // 16-diagonal first level (0 grid: off)
    // the wide level (kWideDiags diagonals, one read pair per wavefront) over what the 16 / 32
    // levels gave up on, before the exact kernel (0 grid: off)
    nw::LaunchCfg wide_fill{}, wide_walk{};
    int64_t wide_pairs = 0, wide_stride = 0;
    int wide_words = 0, wide_lb_cap = 0;
    // seeded band of the current call: reads the 16-diagonal band cannot hold
    // (La - Lb >= 16) go to the wide level centred on their 16-mer hits; seed_pairs widens the
    // wide level's region for them, seed_keys their sort keys
    bool seed_on = false, seed_chunk = false;
    // the seeded list through the second level (32 diagonals, 4 pairs per wavefront) before the wide
    // level, which takes what it leaves (KernelArgs::seed_l2)
    bool seed_l2 = true;
    int64_t seed_pairs = 0;
    int32_t seed_keys = 0;
    int64_t diag16_pass_pairs = 0, diag16_stride = 0;
    DevBuf<uint32_t> d_btab;
    DevBuf<uint32_t> d_sub16;         // exact multi-wave kernel's score rows
    // exact multi-wave kernel on work lists (0 grid: the one-wave kernel, cfg)
    int exact_grid = 0, exact_lds = 0;
    bool exact_tb_lds = true;
    bool exact_full = false;          // long amplicon: every read through the multi-wave kernel
    bool skip16 = false;              // this chunk: the 32-diagonal level only (ops_call's adaptive choice)
    bool exact_small = false;         // this chunk: the exact kernel's work list on a small grid (ops_call)
    bool lane_walk = false;           // resident passes: the first level's lane walk + stop summary (nw_batch_set_lane_walk)
    bool lane_call = false;           // this chunk of ops_call: the lane walk + stop summary (chunks of >= 65536 reads)
    int64_t* zero_ctl = nullptr;      // nw_batch_run_async: classify zeroes the compaction's control block
    // resident passes: the phase events between the kernels (nw_batch_set_phase_events; each timing event
    // recorded between two kernels held the stream ~5-7 us: it writes back the L2's dirty lines)
    bool phase_events = true, phases_recorded = false;
    hipEvent_t ev_h1 = nullptr;       // ops_call: after the last upload (the upload span; ev_in[] do not time)
    int redo_direct = 0;              // this chunk's KernelArgs::redo_direct (launch_range)
    int64_t exact_slab = 0;
    int64_t diag_pass_pairs = 0, diag_stride = 0;
    int diag_words = 0, diag_lb_cap = 0;
    unsigned epoch = 0;               // look-back launches so far (each launch uses a new value)
    int tail_prio = 1;                // KernelArgs::tail_prio
    bool ran = false;
    // ops output (nw_align_ops / nw_batch_set_output(NW_OUT_OPS)): per-read run slots,
    // spill area, compaction scratch; the pipelined call's copy streams and events
    int out_mode = NW_OUT_ROWS;
    int64_t reads_bias = 0;            // kernels index reads with the caller's offsets minus this
    DevBuf<int64_t> d_ctl64, d_opsoff;
    int64_t spill_cap = 0, staging_cap = 0;
    int ops_slot = nw::kOpsSlot;       // runs per read slot (CRISPR_NW_OPS_SLOT: tests force spills)
    int64_t ops_stride = 1;            // reads per slot row (the chunk capacity: ops_reserve)
    hipStream_t s_in = nullptr, s_out = nullptr;
    std::vector<hipEvent_t> ev_in, ev_cs, ev_ce, ev_out, ev_bulk;
    hipEvent_t ev_h0 = nullptr;
    hipEvent_t ev_start = nullptr;     // the second compute stream starts after the first's set-up
    int64_t* h_ctl = nullptr;          // pinned: per chunk ctl[0..3] copied back
    int64_t h_ctl_chunks = 0;
    float ops_h2d_ms = 0.0f, ops_compute_ms = 0.0f;
    bool call_done = false;            // the last operation was nw_align_ops: the getters report its counts
    bool resident_ok = false;          // d_reads / d_offsets hold the last nw_align_ops batch
    // ... or d_packed / d_exc_* / d_offsets (a packed call: classify decodes the reads again)
    bool resident_packed = false;
    int64_t resident_n_exc = 0;
    nw::KernelArgs pkc{};              // the packed-input fields (pk_*) of the chunk launch_range queues next
    // nw_batch_upload_packed: the batch is the 2-bit stream (classify decodes it, writing only
    // the DP reads' bytes); the bytes of every read exist once bytes_full (nw_batch_device_ops)
    bool batch_packed = false, bytes_full = true;
    int64_t batch_pos0 = 0, batch_base0 = 0, batch_nbytes = 0, batch_n_exc = 0;
    int64_t resident_n = 0, resident_lo = 0, resident_hi = 0;
    int64_t call_counts[4] = {0, 0, 0, 0};
    int64_t call_exact = 0;            // reads of the last call that reached the exact kernel
    int64_t ops_h2d_bytes = 0, ops_d2h_bytes = 0;
    // CRISPR_NW_TRACE=1 (diagnostics): an event after every launch of the call's last chunks,
    // printed (us from the first upload) at the end of the call
    bool trace_on = false;
    int trace_chunk = 0;
    // known copies: a resident pass against a new amplicon takes the reads equal to
    // the amplicon the batch was last aligned against (resident_ref: the HDR pass's copies of the
    // reference amplicon) from ONE alignment of that sequence, computed by the exact kernel on the
    // upload stream while the chunks start (d_k*: its bytes, offsets, 2-bit words, record, runs,
    // scratch); KernelArgs::known2 / nw::OpsKnown
    std::string resident_ref;
    std::string known_seq;     // nw_set_known: a sequence whose copies take one alignment in every call
    bool known_on = false;     // the current chunk's known set (kset[kcur]) is prepared
    struct KnownSet {          // one known sequence's alignment (a dual call has one per pass)
        DevBuf<uint8_t> d_kbytes, d_ktb;
        DevBuf<int64_t> d_koff, d_kfb;
        DevBuf<uint32_t> d_k2, d_kslots;
        DevBuf<nw::Stat> d_kstat;
        DevBuf<int32_t> d_kmisc;   // [0] nops, [1..2] ops_ctl, [8..16) fallback counts
        hipEvent_t ev_known = nullptr;
        bool on = false;
        void release() {
            d_kbytes.release(); d_ktb.release(); d_koff.release(); d_kfb.release(); d_k2.release();
            d_kslots.release(); d_kstat.release(); d_kmisc.release();
            if (ev_known) (void)hipEventDestroy(ev_known);
            ev_known = nullptr;
        }
    } kset[2];
    int kcur = 0;
    // a dual call (nw_align_dual_ops_packed_lens): the current chunk's pass writes its records and
    // run offsets at d_stats / d_opsoff + out_off and keeps its running base in ctl block ctl_pass
    int64_t out_off = 0;
    int ctl_pass = 0;
    std::vector<std::pair<std::string, hipEvent_t>> trace_ev;
    size_t trace_used = 0;
};

namespace {

// diagnostics: an event after the launch just queued on c->cs (CRISPR_NW_TRACE)
void tmark(nw_ctx* c, const char* what) {
    if (!c->trace_on) return;
    if (c->trace_used == c->trace_ev.size()) {
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return;
        c->trace_ev.push_back({std::string(), e});
    }
    auto& slot = c->trace_ev[c->trace_used++];
    slot.first = std::to_string(c->trace_chunk) + " " + what;
    (void)hipEventRecord(slot.second, c->cs);
}

int fail(nw_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

// a look-back launch's epoch: new per launch, never 0 (30 bits, nw_common.h lookback_excl)
unsigned next_epoch(nw_ctx* c) {
    c->epoch = (c->epoch + 1) & 0x3fffffffu;
    if (c->epoch == 0) c->epoch = 1;
    return c->epoch;
}

#define HIP_OR_FAIL(ctx, expr)                                                        \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(ctx, e_ == hipErrorOutOfMemory ? NW_E_NOMEM : NW_E_HIP,       \
                        "%s failed: %s", #expr, hipGetErrorString(e_));               \
    } while (0)

// One amplicon's score tables (host side): the int8 profile of the exact kernel and
// the markup bits of the band walk (codes each row scores > 0 against).
struct AmpTables {
    int R = 0;
    std::vector<int8_t> prof;
    std::vector<uint32_t> rowpos;
    std::vector<uint32_t> amp2, seed_key;   // window seeds (Profile::amp2 / seed_key / seed_pos)
    std::vector<uint16_t> seed_pos;
    std::vector<uint32_t> cls;              // classify's LDS image (cls_image)
    bool amp_acgt = false;
};

// classify's LDS image of the amplicon, in the kernel's LDS order: [nd] dwords of the folded
// amplicon (lower-case A C G T, 0 at any other byte and past La), [nd] of its raw bytes (0
// past La), then, with window seeds, amp2, the seed keys and the seed positions (uint16, two
// per word) -- one coalesced copy per block instead of per-byte folding and three table loads.
void cls_image(const std::string& ref, AmpTables* t) {
    const int La = (int)ref.size(), nd = (La + 3) / 4;
    t->cls.assign((size_t)(2 * nd), 0u);
    t->amp_acgt = La > 0;
    for (int q = 0; q < La; ++q) {
        const unsigned char c = (unsigned char)ref[(size_t)q], u = c & 0xDF;
        const bool acgt = u == 'A' || u == 'C' || u == 'G' || u == 'T';
        t->amp_acgt = t->amp_acgt && acgt;
        t->cls[(size_t)(q / 4)] |= (uint32_t)(acgt ? (u | 0x20) : 0) << (8 * (q % 4));
        t->cls[(size_t)(nd + q / 4)] |= (uint32_t)c << (8 * (q % 4));
    }
    if (t->amp2.empty()) return;
    t->cls.insert(t->cls.end(), t->amp2.begin(), t->amp2.end());
    t->cls.insert(t->cls.end(), t->seed_key.begin(), t->seed_key.end());
    for (size_t i = 0; i < t->seed_pos.size(); i += 2)
        t->cls.push_back((uint32_t)t->seed_pos[i] | (i + 1 < t->seed_pos.size() ? (uint32_t)t->seed_pos[i + 1] << 16 : 0u));
}

// The amplicon's 2-bit stream (A C T G = 0 1 2 3 = (byte >> 1) & 3, base p in bits 2 (p % 16)
// of dword p / 16, as nw_pack_reads packs reads; two spare dwords) and its 16-mers of A C G T
// bases only, sorted by (key, position): classify's window seeds.
void seed_tables(const std::string& ref, AmpTables* t) {
    const int La = (int)ref.size();
    if (La < 16 || La > 1024) return;
    t->amp2.assign((size_t)(La + 15) / 16 + 2, 0u);
    std::vector<uint8_t> ok((size_t)La);
    for (int p = 0; p < La; ++p) {
        const unsigned char u = (unsigned char)ref[p] & 0xDF;
        ok[(size_t)p] = u == 'A' || u == 'C' || u == 'G' || u == 'T';
        t->amp2[(size_t)p / 16] |= (uint32_t)(((unsigned char)ref[p] >> 1) & 3u) << (2 * (p % 16));
    }
    std::vector<std::pair<uint32_t, uint16_t>> kp;
    for (int p = 0; p + 16 <= La; ++p) {
        bool all = true;
        uint32_t key = 0;
        for (int b = 0; b < 16; ++b) {
            all = all && ok[(size_t)(p + b)];
            key |= (uint32_t)(((unsigned char)ref[p + b] >> 1) & 3u) << (2 * b);
        }
        if (all) kp.emplace_back(key, (uint16_t)p);
    }
    std::sort(kp.begin(), kp.end());
    for (auto& e : kp) {
        t->seed_key.push_back(e.first);
        t->seed_pos.push_back(e.second);
    }
}

bool amp_tables(const std::string& ref, int scale, AmpTables* t) {
    const int La = (int)ref.size();
    if (La > kMaxRef) return false;
    // markup bits first: an amplicon longer than the one-wave kernels take (R = 0) has
    // only these (the multi-wave kernel aligns it)
    t->rowpos.resize((size_t)La);
    for (int ai = 0; ai < La; ++ai) {
        const uint8_t ca = nw::code_of((unsigned char)ref[ai]);
        uint32_t m = 0;
        for (int code = 0; code < nw::NCODE; ++code)
            if (ca < 16 && code < 16 && nw::kEdna[ca][code] > 0) m |= 1u << code;
        t->rowpos[(size_t)ai] = m;
    }
    const int R = La <= kMaxRefWave ? nw::rows_per_lane_for(La) : 0;
    t->R = R;
    seed_tables(ref, t);
    cls_image(ref, t);
    if (R <= 0) return true;
    const int RP = nw::profile_rp(R);
    t->prof.assign((size_t)nw::NCODE * 64 * RP, 0);
    for (int ai = 0; ai < La; ++ai) {
        const uint8_t ca = nw::code_of((unsigned char)ref[ai]);
        for (int code = 0; code < nw::NCODE; ++code) {
            int s = (ca < 16 && code < 16) ? nw::kEdna[ca][code] * scale : 0;
            t->prof[(size_t)code * 64 * RP + (ai / R) * RP + ai % R] = (int8_t)s;
        }
    }
    return true;
}

// The tables every amplicon shares (they depend on the penalties only): ascii ->
// A T G C N pad/unknown (0..5, 6 = other IUPAC: the band / pair-table alphabet),
// ascii -> EDNAFULL code, and the certified-band score table [amplicon code][read A
// code][read B code] over A T G C N pad, packed int16x2 + 2 * extend.
int upload_shared(nw_ctx* c) {
    const std::string key = std::to_string(c->scale) + "/" + std::to_string(c->gap_extend);
    if (key == c->shared_key && c->d_sub16.p) return NW_OK;
    c->shared_key.clear();
    const int codes6[6] = {0, 1, 2, 3, 14, nw::NCODE_PAD};
    std::vector<uint8_t> lut6(256), lut(256);
    for (int q = 0; q < 256; ++q) {
        const int code = nw::code_of((unsigned char)q);
        int r = 6;
        for (int i = 0; i < 6; ++i)
            if (codes6[i] == code) r = i;
        lut6[(size_t)q] = (uint8_t)r;
        lut[(size_t)q] = (uint8_t)code;
    }
    // amplicon rows by EDNAFULL code (IUPAC amplicons keep the band path), read codes by the
    // 6-code alphabet (reads with other IUPAC codes leave the band: REGION_BAD_*)
    auto sub6 = [&](int cx, int y) {
        const int cy = codes6[y];
        return (cx < 16 && cy < 16) ? nw::kEdna[cx][cy] * c->scale : 0;
    };
    std::vector<uint32_t> btab((size_t)nw::NCODE * 36);
    for (int x = 0; x < nw::NCODE; ++x)
        for (int ya = 0; ya < 6; ++ya)
            for (int yb = 0; yb < 6; ++yb) {
                const uint16_t sa = (uint16_t)(int16_t)(sub6(x, ya) + 2 * c->gap_extend);
                const uint16_t sb = (uint16_t)(int16_t)(sub6(x, yb) + 2 * c->gap_extend);
                btab[(size_t)x * 36 + ya * 6 + yb] = sa | ((uint32_t)sb << 16);
            }
    std::vector<uint32_t> sub16((size_t)nw::NCODE * 4, 0u);
    for (int ca = 0; ca < 16; ++ca)
        for (int code = 0; code < 16; ++code)
            sub16[(size_t)ca * 4 + code / 4] |= (uint32_t)(uint8_t)(int8_t)(nw::kEdna[ca][code] * c->scale)
                                                << (8 * (code % 4));
    HIP_OR_FAIL(c, c->d_sub16.reserve(sub16.size()));
    HIP_OR_FAIL(c, hipMemcpy(c->d_sub16.p, sub16.data(), sub16.size() * 4, hipMemcpyHostToDevice));
    HIP_OR_FAIL(c, c->d_lut6.reserve(256));
    HIP_OR_FAIL(c, c->d_lut.reserve(256));
    HIP_OR_FAIL(c, c->d_btab.reserve(btab.size()));
    HIP_OR_FAIL(c, hipMemcpy(c->d_lut6.p, lut6.data(), 256, hipMemcpyHostToDevice));
    HIP_OR_FAIL(c, hipMemcpy(c->d_lut.p, lut.data(), 256, hipMemcpyHostToDevice));
    HIP_OR_FAIL(c, hipMemcpy(c->d_btab.p, btab.data(), btab.size() * 4, hipMemcpyHostToDevice));
    c->shared_key = key;
    return NW_OK;
}

// Every amplicon's tables in one device arena (one upload): profs[g] points into it.
int upload_profiles(nw_ctx* c, const std::vector<std::string>& refs, std::vector<Profile>* profs) {
    // the tables depend on the amplicons and the score scale
    const std::string key = std::to_string(c->scale);
    if (key == c->arena_key && refs == c->arena_refs && c->d_arena.p) {
        *profs = c->arena_profs;
        return NW_OK;
    }
    c->arena_key.clear();
    std::vector<AmpTables> tabs(refs.size());
    size_t total = 0;
    auto sec = [&](size_t bytes) {
        const size_t at = total;
        total += (bytes + 255) & ~(size_t)255;
        return at;
    };
    struct Off { size_t prof, rowpos, amp, amp2, skey, spos, cls; };
    std::vector<Off> offs(refs.size());
    for (size_t g = 0; g < refs.size(); ++g) {
        if (!amp_tables(refs[g], c->scale, &tabs[g]))
            return fail(c, NW_E_UNSUPPORTED, "amplicon length %d exceeds %d", (int)refs[g].size(), kMaxRef);
        const AmpTables& t = tabs[g];
        const size_t o1 = sec(t.prof.size()), o5 = sec(t.rowpos.size() * 4), o6 = sec(refs[g].size() + 16);
        const size_t o7 = sec(t.amp2.size() * 4), o8 = sec(t.seed_key.size() * 4), o9 = sec(t.seed_pos.size() * 2);
        const size_t o10 = sec(t.cls.size() * 4);
        offs[g] = {o1, o5, o6, o7, o8, o9, o10};
    }
    std::vector<uint8_t> host(std::max<size_t>(total, 256), 0);
    for (size_t g = 0; g < refs.size(); ++g) {
        const AmpTables& t = tabs[g];
        const Off& o = offs[g];
        std::memcpy(host.data() + o.prof, t.prof.data(), t.prof.size());
        std::memcpy(host.data() + o.rowpos, t.rowpos.data(), t.rowpos.size() * 4);
        std::memcpy(host.data() + o.amp, refs[g].data(), refs[g].size());
        std::memcpy(host.data() + o.amp2, t.amp2.data(), t.amp2.size() * 4);
        std::memcpy(host.data() + o.skey, t.seed_key.data(), t.seed_key.size() * 4);
        std::memcpy(host.data() + o.spos, t.seed_pos.data(), t.seed_pos.size() * 2);
        std::memcpy(host.data() + o.cls, t.cls.data(), t.cls.size() * 4);
    }
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));   // no kernel may still read the old arena
    HIP_OR_FAIL(c, c->d_arena.reserve(host.size()));
    HIP_OR_FAIL(c, hipMemcpy(c->d_arena.p, host.data(), host.size(), hipMemcpyHostToDevice));
    profs->resize(refs.size());
    for (size_t g = 0; g < refs.size(); ++g) {
        const Off& o = offs[g];
        uint8_t* b = c->d_arena.p;
        Profile& p = (*profs)[g];
        p.prof = (const int8_t*)(b + o.prof);
        p.rowpos = (const uint32_t*)(b + o.rowpos);
        p.amp = b + o.amp;
        p.R = tabs[g].R;
        p.cls_img = (const uint32_t*)(b + o.cls);
        p.cls_words = (int32_t)tabs[g].cls.size();
        p.amp_acgt = tabs[g].amp_acgt;
        if (!tabs[g].amp2.empty()) {
            p.amp2 = (const uint32_t*)(b + o.amp2);
            p.seed_key = (const uint32_t*)(b + o.skey);
            p.seed_pos = (const uint16_t*)(b + o.spos);
            p.n_seed = (int32_t)tabs[g].seed_key.size();
        }
    }
    c->arena_refs = refs;
    c->arena_profs = *profs;
    c->arena_key = key;
    return NW_OK;
}

int build_profile(nw_ctx* c) {
    int rc = upload_shared(c);
    if (rc) return rc;
    std::vector<Profile> one;
    if ((rc = upload_profiles(c, {c->ref}, &one))) return rc;
    c->cur = one[0];
    return NW_OK;
}

int ops_reserve(nw_ctx* c, int64_t chunk, int64_t n);

int64_t stride_for(int La, int32_t lb_max) { return ((int64_t)La + lb_max + 15) & ~(int64_t)15; }

// Amplicons longer than the one-wave kernels take (kMaxRefWave < La <= kMaxRef):
// every read through the exact multi-wave kernel (nw_exact.hip), one workgroup per
// read, as many workgroups as the CUs hold.
int configure_long(nw_ctx* c) {
    const int La = (int)c->ref.size();
    c->use_diag = false;
    c->diag16_fill.grid = 0;
    c->cfg = nw::LaunchCfg{};
    c->exact_tb_lds = true;
    c->exact_lds = nw::exact_lds_bytes(La, c->lb_max, true);
    c->exact_slab = 0;
    const int W = nw::exact_waves(La);
    int per_cu = std::max(1, 32 / W);   // 32 wavefronts per CU
    if (c->exact_lds > kMaxLds) {
        c->exact_tb_lds = false;
        c->exact_lds = nw::exact_lds_bytes(La, c->lb_max, false);
        c->exact_slab = (nw::exact_slab_bytes(La, c->lb_max) + 255) & ~(int64_t)255;
    }
    if (c->exact_lds <= 0 || c->exact_lds > kMaxLds)
        return fail(c, NW_E_UNSUPPORTED, "reads of %d bases do not fit the kernel for a %d bp amplicon", c->lb_max, La);
    per_cu = std::max(1, std::min(per_cu, kMaxLds / c->exact_lds));
    int64_t grid = std::max<int64_t>(1, std::min<int64_t>((int64_t)c->num_cus * per_cu, std::max<int64_t>(c->n, 1)));
    if (!c->exact_tb_lds) {
        grid = std::max<int64_t>(1, std::min<int64_t>(grid, (2ll << 30) / c->exact_slab));
        HIP_OR_FAIL(c, c->s->d_tb.reserve((size_t)(c->exact_slab * grid)));
    }
    c->exact_grid = (int)grid;
    c->exact_full = true;
    HIP_OR_FAIL(c, c->s->d_fallback.reserve((size_t)std::max<int64_t>(c->n, 1)));
    HIP_OR_FAIL(c, c->s->d_fallback_count.reserve(16));
    return NW_OK;
}

int configure(nw_ctx* c) {
    const int La = (int)c->ref.size();
    const int R = c->cur.R;
    c->exact_full = false;
    if (R <= 0) return configure_long(c);
    // full-storage kernel: every alignment (band disabled) or only the fallbacks
    nw::LaunchCfg cfg{};
    cfg.R = R;
    cfg.tb_mode = nw::TB_GLOBAL_FULL;
    cfg.wpb = 4;
    for (int wpb : {4, 2, 1}) {
        int b = nw::lds_bytes_for(R, La, c->lb_max, nw::TB_LDS_FULL, wpb);
        if (b > 0 && b <= kMaxLds) {
            cfg.tb_mode = nw::TB_LDS_FULL;
            cfg.wpb = wpb;
            cfg.lds_bytes = b;
            break;
        }
    }
    // Traceback in HBM instead of LDS when the LDS traceback leaves a SIMD without a second
    // wavefront (a read's whole matrix at 4 bits per cell: 151 x 280 C1-shape reads take 41 KB per
    // wavefront, three per CU): a lone wavefront issues a VALU instruction per ~4 cycles and
    // waits out its own latencies.  CRISPR_NW_EXACT=lds keeps the LDS traceback (A/Bs).
    const char* ex_env = std::getenv("CRISPR_NW_EXACT");   // "multi[:grid]" | "lds" (tests, A/Bs)
    if (cfg.tb_mode == nw::TB_LDS_FULL && !(ex_env && std::strcmp(ex_env, "lds") == 0) &&
        cfg.wpb * std::min(8, kMaxLds / cfg.lds_bytes) < 8) {
        cfg.tb_mode = nw::TB_GLOBAL_FULL;
        cfg.wpb = 4;
    }
    if (cfg.tb_mode == nw::TB_GLOBAL_FULL) cfg.lds_bytes = nw::lds_bytes_for(R, La, c->lb_max, nw::TB_GLOBAL_FULL, cfg.wpb);
    if (cfg.lds_bytes <= 0 || cfg.lds_bytes > kMaxLds)
        return fail(c, NW_E_UNSUPPORTED, "reads of %d bases do not fit the kernel", c->lb_max);
    int per_cu = std::max(1, std::min(8, kMaxLds / cfg.lds_bytes));
    cfg.grid = c->num_cus * per_cu;
    if (cfg.tb_mode == nw::TB_GLOBAL_FULL) {
        const int64_t per_wave = nw::tb_bytes_per_wave(R, c->lb_max);
        HIP_OR_FAIL(c, c->s->d_tb.reserve((size_t)per_wave * cfg.grid * cfg.wpb));
    }
    c->cfg = cfg;
    // exact multi-wave kernel for the work lists (the reads no band certifies)
    c->exact_grid = 0;
    // Off by default: at the ~15 reads per 1M C2 reads it is not faster than the one-wave
    // kernel (both are VALU-issue bound), so it serves the long amplicons
    const char* ex = ex_env;   // "multi[:grid]": fallbacks through it (tests)
    if (nw::exact_rows_per_lane(La) > 0 && ex && std::strncmp(ex, "multi", 5) == 0) {
        c->exact_tb_lds = true;
        c->exact_lds = nw::exact_lds_bytes(La, c->lb_max, true);
        c->exact_slab = 0;
        int grid = c->num_cus;
        if (c->exact_lds > kMaxLds) {
            c->exact_tb_lds = false;
            c->exact_lds = nw::exact_lds_bytes(La, c->lb_max, false);
            c->exact_slab = (nw::exact_slab_bytes(La, c->lb_max) + 255) & ~(int64_t)255;
            grid = (int)std::max<int64_t>(1, std::min<int64_t>(grid, (1ll << 30) / std::max<int64_t>(c->exact_slab, 1)));
            HIP_OR_FAIL(c, c->s->d_tb.reserve((size_t)(c->exact_slab * grid)));
        }
        if (ex[5] == ':') grid = std::max(1, std::min(grid, std::atoi(ex + 6)));   // split the list between the kernels
        if (c->exact_lds > 0 && c->exact_lds <= kMaxLds) c->exact_grid = grid;
    }
    // -endweight: the band certificate assumes free end gaps; every read goes through
    // the exact kernel (nw_align_kernel), which takes both
    if (c->end_weight) {
        c->use_diag = false;
        c->diag16_fill.grid = 0;
        HIP_OR_FAIL(c, c->s->d_fallback.reserve((size_t)std::max<int64_t>(c->n, 1)));
        HIP_OR_FAIL(c, c->s->d_fallback_count.reserve(16));
        return NW_OK;
    }
    const char* kern = std::getenv("CRISPR_NW_KERNEL");   // "diag" (default) | "diag32" | "full" (tests)
    // certified diagonal band (default): scores and biases within int16, amplicon
    // within the band table's alphabet, non-negative gap costs (the certificate)
    c->use_diag = false;
    const bool want_diag = !kern || std::strncmp(kern, "diag", 4) == 0;
    const int64_t diag_hi = 5ll * c->scale * La + (int64_t)c->gap_extend * (2 * La + 300) + c->gap_open;
    if (want_diag && La <= 1024 && diag_hi < 15000 && c->gap_extend >= 0 &&
        c->gap_open >= c->gap_extend) {
        const int64_t pairs = (c->n + 2) / 2;   // (the second level's list may hold one hole)
        int64_t cap_bytes = 16ll << 30;
        if (const char* rb = std::getenv("CRISPR_NW_REGION_MB")) cap_bytes = std::max(1ll, std::atoll(rb)) << 20;
        c->diag_lb_cap = La + nw::kBandDiags - 1;
        c->diag_words = nw::band_region_words(La, c->lb_max);
        // one level: fill + walk launch configs, region stride and pairs per pass
        // (the wide level at 8, 2 or 4 wavefronts per fill block measured slower or no faster)
        const int wide_fill_wpb = 1, wide_walk_wpb = 2;
        auto level = [&](int W, nw::LaunchCfg& f, nw::LaunchCfg& w, int64_t& stride, int64_t& pass_pairs,
                         int64_t max_pairs = INT64_MAX) -> int {
            f = nw::LaunchCfg{};
            w = nw::LaunchCfg{};
            f.R = w.R = R;
            f.tb_mode = w.tb_mode = nw::TB_DIAG;
            // the wide level aligns few reads, latency-bound: one wavefront per block (fill) and
            // two (walk) spread them over the CUs instead of stacking 8 on a CU's 4 SIMDs
            const bool wide = W > nw::kBandDiags;
            f.wpb = wide ? wide_fill_wpb : 8;
            w.wpb = wide ? wide_walk_wpb : 8;
            f.lds_bytes = nw::band_fill_lds_bytes(La, f.wpb, W);
            w.lds_bytes = nw::band_walk_lds_bytes(La, w.wpb, c->lb_max, W);
            int fb = 0, wb = 0;
            if (f.lds_bytes > kMaxLds || w.lds_bytes > kMaxLds) return 0;
            if (nw::band_occupancy(W, f.wpb, w.wpb, f.lds_bytes, w.lds_bytes, &fb, &wb) != hipSuccess || fb <= 0 ||
                wb <= 0)
                return 0;
            const int ppw = W == 16 ? 8 : (W == 32 ? 4 : 1);   // read pairs per wavefront
            stride = nw::band_region_bytes(La, c->lb_max, W);
            pass_pairs = std::max<int64_t>(ppw, std::min<int64_t>(std::min(pairs, max_pairs), cap_bytes / stride));
            pass_pairs = (pass_pairs + ppw - 1) / ppw * ppw;
            const int64_t pp = std::min<int64_t>(std::max<int64_t>(pairs, 1), pass_pairs);
            f.grid = (int)std::max<int64_t>(1, std::min<int64_t>(((pp + ppw - 1) / ppw + f.wpb - 1) / f.wpb,
                                                                 (int64_t)c->num_cus * fb));
            w.grid = (int)std::max<int64_t>(1, std::min<int64_t>((2 * pp + w.wpb - 1) / w.wpb, (int64_t)c->num_cus * wb));
            return 1;
        };
        const bool use16 = !(kern && std::strcmp(kern, "diag32") == 0) &&
                           level(16, c->diag16_fill, c->diag16_walk, c->diag16_stride, c->diag16_pass_pairs);
        if (!use16) c->diag16_fill.grid = 0;
        if (level(32, c->diag_fill, c->diag_walk, c->diag_stride, c->diag_pass_pairs)) {
            int64_t rbytes = std::max(std::min<int64_t>(std::max<int64_t>(pairs, 1), c->diag_pass_pairs) * c->diag_stride,
                                      use16 ? std::min<int64_t>(std::max<int64_t>(pairs, 1), c->diag16_pass_pairs) *
                                                  c->diag16_stride : 0);
            // the wide level: at most kWidePairs read pairs per chunk in the region (the rest of
            // its list goes to the exact kernel); CRISPR_NW_WIDE=0: off
            c->wide_fill.grid = 0;
            const char* wv = std::getenv("CRISPR_NW_WIDE");
            if (!(wv && std::atoi(wv) == 0) &&
                level(nw::kWideDiags, c->wide_fill, c->wide_walk, c->wide_stride, c->wide_pairs,
                      kWidePairs + c->seed_pairs)) {
                c->wide_words = nw::band_region_words(La, c->lb_max, nw::kWideDiags);
                c->wide_lb_cap = La + nw::kWideDiags - 1;
                rbytes = std::max(rbytes, c->wide_pairs * c->wide_stride);
                HIP_OR_FAIL(c, c->s->d_fallback2.reserve((size_t)std::max<int64_t>(c->n, 1)));
            } else {
                c->wide_fill.grid = 0;
            }
            HIP_OR_FAIL(c, c->s->d_bregion.reserve((size_t)rbytes));
            HIP_OR_FAIL(c, c->s->d_order.reserve((size_t)std::max<int64_t>(c->n, 1)));
            HIP_OR_FAIL(c, c->s->d_redo.reserve((size_t)std::max<int64_t>(c->n, 1)));
            HIP_OR_FAIL(c, c->s->d_redo_flags.reserve((size_t)std::max<int64_t>(c->n, 1)));
            HIP_OR_FAIL(c, c->s->d_lb.reserve((size_t)nw::band_lookback_words(c->n)));
            HIP_OR_FAIL(c, c->s->d_sort_key.reserve((size_t)std::max<int64_t>(c->n, 1)));
            // 64 entries per classify wavefront: 4 per block of 256 reads, ceil(n / 256) + 1 blocks
            HIP_OR_FAIL(c, c->s->d_cert_q.reserve((size_t)std::max<int64_t>(c->n, 1) + 1024));
            HIP_OR_FAIL(c, c->s->d_cert_cnt.reserve((size_t)std::max<int64_t>(c->n, 1) / 64 + 16));
            if (c->seed_on) {
                HIP_OR_FAIL(c, c->s->d_seed.reserve((size_t)std::max<int64_t>(c->n, 1)));
                HIP_OR_FAIL(c, c->s->d_seed2.reserve((size_t)std::max<int64_t>(c->n, 1)));
                // the segment sort pads each 4096-read segment's seeded list to an even length (one
                // entry per segment at most): the list, its flags and its compaction hold n + n/4096 + 2
                const size_t nseed = (size_t)(c->n + c->n / 4096 + 2);
                HIP_OR_FAIL(c, c->s->d_seed_list.reserve(nseed));
                HIP_OR_FAIL(c, c->s->d_seed_flags.reserve(nseed));
                HIP_OR_FAIL(c, c->s->d_seed_list2.reserve(nseed));
            }
            c->use_diag = true;
        }
    }
    HIP_OR_FAIL(c, c->s->d_fallback.reserve((size_t)std::max<int64_t>(c->n, 1)));
    HIP_OR_FAIL(c, c->s->d_fallback_count.reserve(16));
    return NW_OK;
}

}  // namespace

extern "C" {

int nw_create(int device, nw_ctx** out) {
    if (!out) return NW_E_INVALID;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return NW_E_HIP;
    if (device < 0 || device >= count) return NW_E_INVALID;
    nw_ctx* c = new nw_ctx();
    c->device = device;
    // Creation order decides which streams share a hardware queue (a process gets
    // GPU_MAX_HW_QUEUES = 4; the fifth stream shares the first one's queue, and a queue runs
    // its packets in order, so a cross-stream wait queued there holds back the other
    // stream too).  Default: s_in first and the third compute stream (the pipelined call's
    // tail stream) last, so those two share: the uploads of a call are all queued before its
    // first tail packet.  (Round 2's order, where s_out shared the first compute stream's
    // queue: 2.475 vs 2.423 ms per 1M-read call.)
    hipStream_t* order[5] = {&c->s_in, &c->stream, &c->cstream[1], &c->s_out, &c->cstream[2]};
    bool streams_ok = hipSetDevice(device) == hipSuccess;
    for (hipStream_t* sp : order)
        streams_ok = streams_ok && hipStreamCreateWithFlags(sp, hipStreamNonBlocking) == hipSuccess;
    if (!streams_ok || hipEventCreate(&c->ev_h0) != hipSuccess ||
        hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming) != hipSuccess ||
        hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
        hipEventCreate(&c->ev_fill) != hipSuccess || hipEventCreate(&c->ev_walk) != hipSuccess ||
        hipEventCreate(&c->ev_sort) != hipSuccess || hipEventCreate(&c->ev_l2) != hipSuccess ||
        hipEventCreate(&c->ev_h1) != hipSuccess) {
        delete c;
        return NW_E_HIP;
    }
    c->cs = c->stream;
    c->cstream[0] = c->stream;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) == hipSuccess && prop.multiProcessorCount > 0)
        c->num_cus = prop.multiProcessorCount;
    *out = c;
    return NW_OK;
}

void nw_destroy(nw_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->d_arena.release(); c->d_lut.release();
    c->d_reads.release(); c->d_offsets.release(); c->d_out.release();
    c->d_packed.release(); c->d_exc_byte.release(); c->d_exc_pos.release(); c->d_lens.release();
    c->d_stats.release();
    c->d_lut6.release();
    c->d_btab.release();
    c->d_sub16.release();
    for (Scratch& S : c->sc) S.release();
    c->d_ctl64.release(); c->d_opsoff.release();
    if (c->s_in) (void)hipStreamSynchronize(c->s_in);
    for (auto& ks : c->kset) ks.release();
    for (auto& t : c->trace_ev) (void)hipEventDestroy(t.second);
    for (hipEvent_t e : c->ev_bulk) (void)hipEventDestroy(e);
    for (int k = 1; k < kComputeStreams; ++k)
        if (c->cstream[k]) (void)hipStreamSynchronize(c->cstream[k]);
    if (c->s_out) (void)hipStreamSynchronize(c->s_out);
    for (auto* v : {&c->ev_in, &c->ev_cs, &c->ev_ce, &c->ev_out})
        for (hipEvent_t e : *v) (void)hipEventDestroy(e);
    if (c->h_ctl) (void)hipHostFree(c->h_ctl);
    if (c->h_lens) (void)hipHostFree(c->h_lens);
    if (c->ev_h0) (void)hipEventDestroy(c->ev_h0);
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->s_in) (void)hipStreamDestroy(c->s_in);
    for (int k = 1; k < kComputeStreams; ++k)
        if (c->cstream[k]) (void)hipStreamDestroy(c->cstream[k]);
    if (c->s_out) (void)hipStreamDestroy(c->s_out);
    if (c->ev_fill) (void)hipEventDestroy(c->ev_fill);
    if (c->ev_h1) (void)hipEventDestroy(c->ev_h1);
    if (c->ev_sort) (void)hipEventDestroy(c->ev_sort);
    if (c->ev_l2) (void)hipEventDestroy(c->ev_l2);
    if (c->ev_walk) (void)hipEventDestroy(c->ev_walk);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

const char* nw_last_error(const nw_ctx* c) { return c ? c->err.c_str() : "null context"; }

int nw_set_params(nw_ctx* c, float gap_open, float gap_extend, int end_weight, float end_open,
                  float end_extend, const char* matrix, int tie_policy) {
    if (!c) return NW_E_INVALID;
    if (matrix && *matrix) {
        std::string m(matrix);
        for (auto& ch : m) ch = (char)std::toupper((unsigned char)ch);
        if (m != "EDNAFULL") return fail(c, NW_E_UNSUPPORTED, "matrix %s not supported (EDNAFULL only)", matrix);
    }
    if (tie_policy != NW_TIE_EMBOSS) return fail(c, NW_E_UNSUPPORTED, "tie policy %d not supported", tie_policy);
    if (!(gap_open >= 0.0f) || !(gap_extend >= 0.0f) || gap_open > 1000.0f || gap_extend > 1000.0f)
        return fail(c, NW_E_INVALID, "gap penalties out of range: %g %g", gap_open, gap_extend);
    if (end_weight && (!(end_open >= 0.0f) || !(end_extend >= 0.0f) || end_open > 1000.0f || end_extend > 1000.0f))
        return fail(c, NW_E_INVALID, "end gap penalties out of range: %g %g", end_open, end_extend);
    int scale = 0;
    for (int s = 1; s <= 16; s *= 2) {
        double o = (double)gap_open * s, e = (double)gap_extend * s;
        double eo = end_weight ? (double)end_open * s : 0.0, ee = end_weight ? (double)end_extend * s : 0.0;
        if (o == std::floor(o) && e == std::floor(e) && eo == std::floor(eo) && ee == std::floor(ee)) {
            scale = s;
            break;
        }
    }
    if (!scale) return fail(c, NW_E_INEXACT, "gap penalties %g/%g (end %g/%g) are not multiples of 1/16", gap_open,
                            gap_extend, end_open, end_extend);
    c->gap_open_f = gap_open;
    c->gap_extend_f = gap_extend;
    c->scale = scale;
    c->gap_open = (int)std::lround((double)gap_open * scale);
    c->gap_extend = (int)std::lround((double)gap_extend * scale);
    c->end_weight = end_weight != 0;
    c->end_open = end_weight ? (int)std::lround((double)end_open * scale) : 0;
    c->end_extend = end_weight ? (int)std::lround((double)end_extend * scale) : 0;
    if (!c->ref.empty()) {
        (void)hipSetDevice(c->device);
        return build_profile(c);
    }
    return NW_OK;
}

int nw_score_scale(const nw_ctx* c) { return c ? c->scale : 0; }

int nw_set_reference(nw_ctx* c, const char* ref, int32_t ref_len) {
    if (!c || !ref || ref_len <= 0) return fail(c, NW_E_INVALID, "empty amplicon");
    if (ref_len > kMaxRef) return fail(c, NW_E_UNSUPPORTED, "amplicon length %d exceeds %d", ref_len, kMaxRef);
    (void)hipSetDevice(c->device);
    c->ref.assign(ref, ref + ref_len);
    c->ran = false;
    c->call_done = false;
    return build_profile(c);
}

int64_t nw_required_stride(const nw_ctx* c, int32_t max_read_len) {
    if (!c || c->ref.empty()) return 0;
    return stride_for((int)c->ref.size(), std::max(max_read_len, 1));
}

int nw_batch_upload(nw_ctx* c, const char* reads, const int64_t* offsets, int64_t n) {
    if (!c) return NW_E_INVALID;
    if (c->ref.empty()) return fail(c, NW_E_STATE, "nw_set_reference must come first");
    if (n < 0 || (n > 0 && (!offsets || !reads))) return fail(c, NW_E_INVALID, "bad batch");
    (void)hipSetDevice(c->device);
    const int La = (int)c->ref.size();
    int32_t lb_max = 1;
    int64_t cells = 0;
    c->read_lens.resize((size_t)n);
    for (int64_t r = 0; r < n; ++r) {
        const int64_t len = offsets[r + 1] - offsets[r];
        if (len < 0 || len > (1 << 20)) return fail(c, NW_E_INVALID, "read %lld has length %lld", (long long)r, (long long)len);
        c->read_lens[(size_t)r] = (int32_t)len;
        lb_max = std::max<int32_t>(lb_max, (int32_t)len);
        cells += (int64_t)La * len;
    }
    const int64_t base = n ? offsets[0] : 0;
    const int64_t nbytes = n ? offsets[n] - base : 0;
    std::vector<int64_t> rel((size_t)n + 1);
    for (int64_t r = 0; r <= n; ++r) rel[(size_t)r] = n ? offsets[r] - base : 0;
    c->n = n;
    c->lb_max = lb_max;
    c->cells = cells;
    c->stride = stride_for(La, lb_max);
    HIP_OR_FAIL(c, c->d_reads.reserve((size_t)nbytes + 512));   // the walk DMAs whole 256-B chunks
    HIP_OR_FAIL(c, c->d_offsets.reserve((size_t)n + 1));
    if (c->out_mode == NW_OUT_ROWS) HIP_OR_FAIL(c, c->d_out.reserve((size_t)std::max<int64_t>(n, 1) * 3 * c->stride));
    HIP_OR_FAIL(c, c->d_stats.reserve((size_t)std::max<int64_t>(n, 1)));
    c->resident_ok = false;
    c->batch_packed = false;
    c->bytes_full = true;
    c->pkc = nw::KernelArgs{};
    if (nbytes) HIP_OR_FAIL(c, hipMemcpyAsync(c->d_reads.p, reads + base, (size_t)nbytes, hipMemcpyHostToDevice, c->stream));
    HIP_OR_FAIL(c, hipMemcpyAsync(c->d_offsets.p, rel.data(), sizeof(int64_t) * (size_t)(n + 1), hipMemcpyHostToDevice, c->stream));
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    c->reads_bias = 0;
    int rc = configure(c);
    if (rc) return rc;
    if (c->out_mode == NW_OUT_OPS && (rc = ops_reserve(c, n, n))) return rc;
    c->ran = false;
    c->call_done = false;
    return NW_OK;
}

int nw_batch_upload_packed(nw_ctx* c, const uint8_t* packed, const int64_t* offsets, const uint16_t* lens, int64_t n,
                           const int64_t* exc_pos, const uint8_t* exc_byte, int64_t n_exc) {
    if (!c) return NW_E_INVALID;
    if (c->ref.empty()) return fail(c, NW_E_STATE, "nw_set_reference must come first");
    if (c->out_mode != NW_OUT_OPS) return fail(c, NW_E_STATE, "a packed batch needs nw_batch_set_output(NW_OUT_OPS)");
    if (n <= 0 || !offsets || !packed || !lens || (n_exc > 0 && (!exc_pos || !exc_byte)) || n_exc < 0)
        return fail(c, NW_E_INVALID, "bad batch");
    (void)hipSetDevice(c->device);
    const int La = (int)c->ref.size();
    int32_t lb_max = 1;
    int64_t cells = 0;
    c->read_lens.resize((size_t)n);
    for (int64_t r = 0; r < n; ++r) {
        const int64_t len = offsets[r + 1] - offsets[r];
        if (len < 0 || len > 65535 || len != lens[r])
            return fail(c, NW_E_INVALID, "read %lld: length %lld, lens %u", (long long)r, (long long)len, (unsigned)lens[r]);
        c->read_lens[(size_t)r] = (int32_t)len;
        lb_max = std::max<int32_t>(lb_max, (int32_t)len);
        cells += (int64_t)La * len;
    }
    const int64_t base0 = offsets[0], nbytes = offsets[n] - base0;
    const int64_t P0 = (base0 / 16) * 4, pk_hi = (offsets[n] + 3) / 4, q0 = base0 / 4;
    const int64_t ngroups = n / nw::kLenGroup + 1;
    c->n = n;
    c->lb_max = lb_max;
    c->cells = cells;
    c->stride = stride_for(La, lb_max);
    HIP_OR_FAIL(c, c->d_reads.reserve((size_t)nbytes + 512 + 16));
    HIP_OR_FAIL(c, c->d_offsets.reserve((size_t)n + 1));
    HIP_OR_FAIL(c, c->d_stats.reserve((size_t)n));
    HIP_OR_FAIL(c, c->d_packed.reserve((size_t)(pk_hi - P0) + 64));
    HIP_OR_FAIL(c, c->d_exc_pos.reserve((size_t)std::max<int64_t>(n_exc, 1)));
    HIP_OR_FAIL(c, c->d_exc_byte.reserve((size_t)std::max<int64_t>(n_exc, 1)));
    HIP_OR_FAIL(c, c->d_lens.reserve((size_t)(8 * ngroups + 2 * n + 64)));
    std::vector<int64_t> gb((size_t)ngroups);
    for (int64_t g = 0; g < ngroups; ++g) gb[(size_t)g] = offsets[g * nw::kLenGroup];
    c->resident_ok = false;
    HIP_OR_FAIL(c, hipMemcpyAsync(c->d_packed.p + (q0 - P0), packed + q0, (size_t)(pk_hi - q0), hipMemcpyHostToDevice,
                                  c->stream));
    if (n_exc) {
        HIP_OR_FAIL(c, hipMemcpyAsync(c->d_exc_pos.p, exc_pos, 8 * (size_t)n_exc, hipMemcpyHostToDevice, c->stream));
        HIP_OR_FAIL(c, hipMemcpyAsync(c->d_exc_byte.p, exc_byte, (size_t)n_exc, hipMemcpyHostToDevice, c->stream));
    }
    HIP_OR_FAIL(c, hipMemcpyAsync(c->d_lens.p, gb.data(), 8 * (size_t)ngroups, hipMemcpyHostToDevice, c->stream));
    HIP_OR_FAIL(c, hipMemcpyAsync(c->d_lens.p + 8 * ngroups, lens, 2 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    c->reads_bias = base0 & ~(int64_t)15;
    int rc = configure(c);
    if (rc) return rc;
    if ((rc = ops_reserve(c, n, n))) return rc;
    c->batch_packed = true;
    c->batch_pos0 = 4 * P0;
    c->batch_base0 = base0;
    c->batch_nbytes = nbytes;
    c->batch_n_exc = n_exc;
    c->pkc = nw::KernelArgs{};
    nw::LenSeg ls{(const uint16_t*)(c->d_lens.p + 8 * ngroups), (const int64_t*)c->d_lens.p, 0, ngroups, 0, n,
                  c->d_offsets.p};
    if (c->use_diag) {   // classify decodes the batch on every run (KernelArgs::pk_*)
        c->pkc.pk_words = (const uint32_t*)c->d_packed.p;
        c->pkc.pk_pos0 = 4 * P0;
        c->pkc.pk_exc_pos = c->d_exc_pos.p;
        c->pkc.pk_exc_byte = c->d_exc_byte.p;
        c->pkc.pk_e0 = 0;
        c->pkc.pk_e1 = n_exc;
        c->pkc.pk_len = ls.len;
        c->pkc.pk_gbase = ls.gbase;
        c->pkc.pk_call_lo = 0;
        c->bytes_full = false;
    } else {   // the exact kernels read bytes: unpack once
        HIP_OR_FAIL(c, nw::launch_unpack((const uint32_t*)c->d_packed.p, P0, base0, offsets[n], c->d_exc_pos.p,
                                         c->d_exc_byte.p, 0, n_exc, c->d_reads.p, c->reads_bias, c->stream, &ls));
        HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
        c->bytes_full = true;
    }
    c->ran = false;
    c->call_done = false;
    return NW_OK;
}

}  // extern "C"

namespace {

// The exact int32 kernel over a device work list (a.work_list / a.work_count): the
// multi-wave kernel (nw_exact.hip) when configured, else the one-wave kernel.
// Entries [0, exact_grid) go to the multi-wave kernel (one read per workgroup: the
// latency of a few reads), the rest, if any, to the one-wave kernel (throughput when
// many reads need the exact DP, e.g. an unrelated amplicon's HDR pass).
hipError_t launch_work(nw_ctx* c, const nw::KernelArgs& a) {
    // a work list expected short (ops_call: the recent chunks sent few reads to the exact
    // kernel): a small grid, so that the launch's empty blocks do not wait behind the other
    // chunks' kernels for LDS (a full grid of early-exiting blocks measured ~20 us per chunk)
    nw::LaunchCfg cfg = c->cfg;
    if (a.work_list && c->exact_small) cfg.grid = std::min(cfg.grid, std::max(1, c->num_cus / 2));
    if (c->exact_grid <= 0) return nw::launch(a, cfg, c->cs);
    hipError_t e = nw::launch_exact(a, c->exact_grid, c->exact_lds, c->exact_tb_lds, c->exact_slab, true, c->cs);
    if (e != hipSuccess) return e;
    nw::KernelArgs rest = a;
    rest.work_lo = c->exact_grid;
    return nw::launch(rest, c->cfg, c->cs);
}

// Launches the kernels for the c->n reads that start at read `base` of the
// uploaded arrays (outputs, records and fallback queue at the same index).
// Everything is queued on c->stream; nothing synchronises.
int launch_range(nw_ctx* c, int64_t base) {
    c->tail_prio = true;   // the latency-bound kernels of a chunk's chain at raised issue priority (-1.1 %)
    nw::KernelArgs a{};
    a.reads = c->d_reads.p - c->reads_bias;
    a.offsets = c->d_offsets.p + base;
    a.n = c->n;
    a.prof = c->cur.prof;
    a.lut6 = nullptr;
    a.lut = c->d_lut.p;
    a.amp = c->cur.amp;
    a.La = (int32_t)c->ref.size();
    a.gap_open = c->gap_open;
    a.gap_extend = c->gap_extend;
    a.Lb_max = c->lb_max;
    a.out = c->d_out.p + base * 3 * c->stride;
    a.stride = c->stride;
    a.stats = c->d_stats.p + c->out_off + base;
    a.tb_global = c->s->d_tb.p;
    a.sub16 = c->d_sub16.p;
    a.rowpos = c->cur.rowpos;
    a.end_weight = c->end_weight;
    a.tail_prio = c->tail_prio;
    a.band_summ = (c->lane_walk && c->phases) || c->lane_call ? 1 : 0;   // resident passes, the call's large chunks
    a.end_open = c->end_open;
    a.end_extend = c->end_extend;
    a.tb_wave_bytes = c->cfg.tb_mode == nw::TB_GLOBAL_FULL ? nw::tb_bytes_per_wave(c->cur.R, c->lb_max) : 0;
    a.fallback_list = c->s->d_fallback.p + base;
    a.fallback_count = c->s->d_fallback_count.p;
    if (c->out_mode == NW_OUT_OPS) {
        // runs into chunk-relative slots; rows are not written
        a.out = nullptr;
        a.ops = c->s->d_slots.p;
        a.ops_slot = c->ops_slot;
        a.ops_stride = c->ops_stride;
        a.nops = c->s->d_nops.p;
        a.spill = c->s->d_spill.p;
        a.spill_cap = c->spill_cap;
        a.ops_ctl = c->s->d_opsctl.p;
        // the band path writes every read's run count and zeroes its counters in its
        // first kernel (nw_band_classify): no memset launches in the chunk's chain
        if (!c->use_diag || c->n <= 0) {
            HIP_OR_FAIL(c, hipMemsetAsync(c->s->d_nops.p, 0, sizeof(int32_t) * (size_t)std::max<int64_t>(c->n, 1), c->cs));
            HIP_OR_FAIL(c, hipMemsetAsync(c->s->d_opsctl.p, 0, 2 * sizeof(int32_t), c->cs));
        }
    }
    if (c->use_diag) {
        // length sort, certified band fill + walk per pass, exact int32 kernel on the rest
        if (c->n <= 0) return hipMemsetAsync(c->s->d_fallback_count.p, 0, 16 * sizeof(int32_t), c->cs) == hipSuccess
                                  ? NW_OK : fail(c, NW_E_HIP, "hipMemsetAsync failed");
        a.lut6 = c->d_lut6.p;
        a.band_order = c->s->d_order.p;
        a.band_region = c->s->d_bregion.p;
        a.band_stride = c->diag_stride;
        a.band_words = c->diag_words;
        a.band_lb_cap = c->diag_lb_cap;
        a.band_maxsub = 5 * c->scale;
        a.band_tab = c->d_btab.p;
        a.rowpos = c->cur.rowpos;
        a.sort_key = c->s->d_sort_key.p;
        a.band_count = c->s->d_fallback_count.p + 1;   // the sort writes the DP count here
        a.amp2 = c->cur.amp2;
        a.seed_key = c->cur.seed_key;
        a.seed_pos = c->cur.seed_pos;
        a.n_seed = c->cur.n_seed;
        a.cls_img = c->cur.cls_img;
        a.cls_words = c->cur.cls_words;
        a.amp_acgt = c->cur.amp_acgt ? 1 : 0;
        // seeded band: the packed classify marks the reads, the segment sort lists them apart
        // (sorted by their hits' diagonals), the wide level takes that list after its own
        c->seed_chunk = c->seed_on && c->pkc.pk_words && c->wide_fill.grid > 0 && c->cur.n_seed > 0;
        if (c->seed_chunk) {
            a.seed_info = c->s->d_seed.p;
            a.seed_info2 = c->s->d_seed2.p;
            a.seed_keys = c->seed_keys;
            a.seed_list = c->s->d_seed_list.p;
            a.seed_count = c->s->d_fallback_count.p + 7;   // zeroed by nw_band_classify
        }
        a.lb_status = c->s->d_lb.p;
        // packed input (ops_call): classify decodes the chunk (KernelArgs::pk_*)
        a.pk_words = c->pkc.pk_words;
        a.pk_pos0 = c->pkc.pk_pos0;
        a.pk_exc_pos = c->pkc.pk_exc_pos;
        a.pk_exc_byte = c->pkc.pk_exc_byte;
        a.pk_e0 = c->pkc.pk_e0;
        a.pk_e1 = c->pkc.pk_e1;
        a.pk_len = c->pkc.pk_len;
        a.pk_gbase = c->pkc.pk_gbase;
        a.pk_call_lo = c->pkc.pk_call_lo;
        a.known2 = c->known_on ? c->kset[c->kcur].d_k2.p : nullptr;
        // the three-substitution and one-indel checks on classify's queues (nw_band_cert; packed input,
        // ops output: the only classify that has those certificates)
        if (a.pk_words && a.ops) {
            a.cert_q = c->s->d_cert_q.p;
            a.cert_cnt = c->s->d_cert_cnt.p;
        }
        a.zero_ctl64 = c->zero_ctl;
        a.zero_ctl64_n = nw::kOpsCtlAll;
        HIP_OR_FAIL(c, nw::launch_band_sort(a, next_epoch(c), c->cs));
        tmark(c, "classify+sort");
        const bool pev = c->phases && c->phase_events;   // phase events (resident passes that ask for them)
        if (pev) HIP_OR_FAIL(c, hipEventRecord(c->ev_sort, c->cs));
        const int64_t pairs = (c->n + 2) / 2;   // (the second level's list may hold one hole)
        // level 1 (16 diagonals) over the sorted reads; what it cannot certify -> redo list
        // -> level 2 (32 diagonals) -> the exact int32 kernel.  Kernels clamp the pair
        // ranges to the device-side counts.
        const bool two = c->diag16_fill.grid > 0 && !c->skip16;
        a.redo_list = c->s->d_redo.p;
        a.redo_count = c->s->d_fallback_count.p + 2;
        if (two) a.redo_flags = c->s->d_redo_flags.p;   // the first level's walk writes every position's
        // a chunk whose first level hands on at most `direct` reads skips the second level on
        // the device: the wide level takes them (up to 1/16 of the chunk, as many as its region
        // holds), or without it the exact kernel (1024).  A chunk where more reads need more than
        // 16 diagonals (the HDR pass) keeps the second level, 4 read pairs per wavefront, and the
        // adaptive first-level choice sees them.  CRISPR_NW_DIRECT=0: always both levels.
        int direct = c->wide_fill.grid > 0
                         ? (int)std::max<int64_t>(1024, std::min<int64_t>(c->n / 16, 2 * c->wide_pairs))
                         : 1024;
        if (const char* e = std::getenv("CRISPR_NW_DIRECT")) direct = std::max(0, std::atoi(e));
        if (!two) direct = 0;
        c->redo_direct = direct;
        // a chunk of >= 65536 reads with at most `direct` DP reads (device count) skips the first level too,
        // when the wide level can take them: one level's latency in its chain instead of three (in-process
        // A/B, C2 call 1.849 -> 1.771 ms, outputs identical; C1, C3, C5 unchanged).  Smaller launches (the
        // tests' batches) keep the first level.  CRISPR_NW_L1SKIP=0: off
        {
            const char* e = std::getenv("CRISPR_NW_L1SKIP");
            a.l1_skip = two && c->wide_fill.grid > 0 && c->n >= 65536 && !(e && std::atoi(e) == 0) ? direct : 0;
        }
        for (int lvl = two ? 0 : 1; lvl < 2; ++lvl) {
            nw::KernelArgs al = a;
            al.redo_direct = lvl == 1 ? direct : 0;
            const int W = lvl == 0 ? 16 : 32;
            if (lvl == 1 && two) {
                HIP_OR_FAIL(c, nw::launch_redo_compact(a, c->n, next_epoch(c), c->cs));
                tmark(c, "redo");
                al.band_order = c->s->d_redo.p;
                al.band_count = a.redo_count;
            }
            if (lvl == 1 && c->seed_chunk && c->seed_l2) {   // then the seeded list
                al.seed_l2 = 1;
                al.seed_flags = c->s->d_seed_flags.p;
            }
            al.band_stride = lvl == 0 ? c->diag16_stride : c->diag_stride;
            const int64_t pp = lvl == 0 ? c->diag16_pass_pairs : c->diag_pass_pairs;
            const nw::LaunchCfg& fc = lvl == 0 ? c->diag16_fill : c->diag_fill;
            const nw::LaunchCfg& wc = lvl == 0 ? c->diag16_walk : c->diag_walk;
            const bool first = lvl == (two ? 0 : 1);
            for (int64_t lo = 0; lo < pairs; lo += pp) {
                nw::KernelArgs ap = al;
                ap.band_pair_lo = lo;
                ap.band_pair_hi = std::min(pairs, lo + pp);
                HIP_OR_FAIL(c, nw::launch_band(W, ap, fc, wc, c->cs, pev && first && lo == 0 ? c->ev_fill : nullptr));
                tmark(c, W == 16 ? "fill16+walk16" : "fill32+walk32");
                if (pev && first && lo == 0) HIP_OR_FAIL(c, hipEventRecord(c->ev_walk, c->cs));
            }
            if (first && c->split_to) {   // the latency-bound rest of the chunk on the tail stream
                HIP_OR_FAIL(c, hipEventRecord(c->split_ev, c->cs));
                HIP_OR_FAIL(c, hipStreamWaitEvent(c->split_to, c->split_ev, 0));
                c->cs = c->split_to;
            }
        }
        if (c->seed_chunk && c->seed_l2) {
            // the pairs of seeded reads the 32-diagonal level did not certify both of, compacted in the
            // seeded list's order (the wide level's pairs are that level's pairs: reads of nearby hits,
            // one sort segment): they replace that list (a certified partner is aligned again, the same)
            nw::KernelArgs ac = a;
            ac.band_order = c->s->d_seed_list.p;
            ac.band_count = a.seed_count;
            ac.redo_flags = c->s->d_seed_flags.p;
            ac.l1_skip = 0;
            ac.redo_list = c->s->d_seed_list2.p;
            ac.redo_count = c->s->d_fallback_count.p + 8;   // zeroed by nw_band_classify
            HIP_OR_FAIL(c, nw::launch_redo_compact(ac, c->n + c->n / 4096 + 2, next_epoch(c), c->cs, true));
            tmark(c, "seed compact");
            a.seed_list = ac.redo_list;
            a.seed_count = ac.redo_count;
        }
        if (pev) HIP_OR_FAIL(c, hipEventRecord(c->ev_l2, c->cs));
        a.work_list = a.fallback_list;   // what the 16 / 32 levels could not certify
        a.work_count = c->s->d_fallback_count.p;
        a.redo_direct = direct;
        if (c->wide_fill.grid > 0) {
            // the wide level over that list (and, direct hand-off, the first level's redo list):
            // one read pair per wavefront, 128 diagonals: a few fill + walk launches of ~20 us
            // latency where the exact kernel took ~80 us per chunk; its give-ups -> the exact kernel
            nw::KernelArgs aw = a;
            aw.band_from_work = 1;
            aw.band_count = a.work_count;
            aw.redo_flags = nullptr;
            aw.band_stride = c->wide_stride;
            aw.band_words = c->wide_words;
            aw.band_lb_cap = c->wide_lb_cap;
            aw.band_pair_lo = 0;
            aw.band_pair_hi = c->wide_pairs;
            aw.fallback_list = c->s->d_fallback2.p + base;
            aw.fallback_count = c->s->d_fallback_count.p + 6;   // zeroed by nw_band_classify
            HIP_OR_FAIL(c, nw::launch_band(nw::kWideDiags, aw, c->wide_fill, c->wide_walk, c->cs, nullptr));
            tmark(c, "wide");
            a.work_list = aw.fallback_list;
            a.work_count = aw.fallback_count;
            a.redo_direct = 0;
        }
        HIP_OR_FAIL(c, launch_work(c, a));
        tmark(c, "exact");
        return NW_OK;
    }
    HIP_OR_FAIL(c, hipMemsetAsync(c->s->d_fallback_count.p, 0, 16 * sizeof(int32_t), c->cs));
    if (c->exact_full) {   // long amplicon: every read through the multi-wave kernel
        if (c->n > 0)
            HIP_OR_FAIL(c, nw::launch_exact(a, c->exact_grid, c->exact_lds, c->exact_tb_lds, c->exact_slab, false,
                                            c->cs));
        return NW_OK;
    }
    if (c->n > 0) HIP_OR_FAIL(c, launch_work(c, a));   // every read (null work list)
    return NW_OK;
}


// Ops-mode buffers for chunks of up to `chunk` reads of a call over n reads:
// slots and counts per chunk (reused chunk after chunk, the compaction copies them
// out in-stream), the spill area, and two staging arrays (chunk c compacts into
// staging[c % 2] while the copy of chunk c - 1's runs may still be in flight).
int ops_reserve(nw_ctx* c, int64_t chunk, int64_t n) {
    chunk = std::max<int64_t>(chunk, 1);
    const int64_t spill_mb = 64;
    c->ops_slot = nw::kOpsSlot;
    if (const char* e = std::getenv("CRISPR_NW_OPS_SLOT")) c->ops_slot = std::max(1, std::atoi(e));
    c->spill_cap = (spill_mb << 20) / 4;
    if (const char* e = std::getenv("CRISPR_NW_SPILL_WORDS")) c->spill_cap = std::max(1ll, std::atoll(e));   // tests
    c->staging_cap = chunk * c->ops_slot + c->spill_cap;
    c->ops_stride = chunk;
    HIP_OR_FAIL(c, c->s->d_slots.reserve((size_t)(2 * chunk * c->ops_slot)));   // column-major + row-major areas
    HIP_OR_FAIL(c, c->s->d_nops.reserve((size_t)chunk));
    HIP_OR_FAIL(c, c->s->d_spill.reserve((size_t)c->spill_cap));
    HIP_OR_FAIL(c, c->s->d_opsctl.reserve(2));
    HIP_OR_FAIL(c, c->d_ctl64.reserve(2 * nw::kOpsCtlAll));   // a dual call: one block per pass
    HIP_OR_FAIL(c, c->s->d_lb.reserve((size_t)nw::band_lookback_words(chunk)));
    HIP_OR_FAIL(c, c->d_opsoff.reserve((size_t)std::max<int64_t>(n, 1) + 1));
    HIP_OR_FAIL(c, c->s->d_staging.reserve((size_t)c->staging_cap));
    return NW_OK;
}

// Kernels of c->n reads starting at read `base`, then their compaction into
// staging[which]: ops_off of those reads (global: the call's running base in
// ctl[0]) and ctl[1..3] = chunk base, chunk total, error.
int launch_range_ops(nw_ctx* c, int64_t base, hipEvent_t staging_free = nullptr, hipEvent_t prev_done = nullptr,
                     int64_t* hctl = nullptr, int parity = 0, const nw::OpsHostOut* host = nullptr) {
    int rc = launch_range(c, base);
    if (rc) return rc;
    // only the compaction writes the set's staging array: it waits for the copy of the
    // runs it held two chunks ago, and (the running base of ctl) for the previous
    // chunk's compaction on the other stream; the kernels before it wait for neither
    if (staging_free) HIP_OR_FAIL(c, hipStreamWaitEvent(c->cs, staging_free, 0));
    if (prev_done) HIP_OR_FAIL(c, hipStreamWaitEvent(c->cs, prev_done, 0));
    nw::OpsCounts cnt{};
    cnt.fallback = c->s->d_fallback_count.p;
    cnt.prio = c->tail_prio;
    if (c->use_diag && c->n > 0) {
        cnt.band = c->s->d_fallback_count.p + 1;
        // second-level reads of a two-level chunk; a chunk run on the 32-diagonal level alone
        // counts its DP reads apart (ctl[7]: the adaptive choice reads two-level chunks only)
        if (c->diag16_fill.grid > 0 && !c->skip16) cnt.redo = c->s->d_fallback_count.p + 2;
        cnt.one_level = c->diag16_fill.grid > 0 && c->skip16;
        cnt.direct = c->skip16 ? 0 : c->redo_direct;
        if (c->wide_fill.grid > 0) cnt.exact = c->s->d_fallback_count.p + 6;
        if (c->seed_chunk) {
            cnt.seeded = c->s->d_fallback_count.p + 7;
            cnt.seed_pad = c->s->d_fallback_count.p + 9;   // the sort's padding entries (zeroed by classify)
        }
        if (c->seed_chunk && c->seed_l2) cnt.seeded_l2 = c->s->d_fallback_count.p + 8;
    }
    if (c->n <= 0) cnt.fallback = nullptr;
    nw::OpsKnown kn{};
    if (c->known_on) {   // the known alignment (computed on the upload stream) before any copy takes it
        auto& K = c->kset[c->kcur];
        HIP_OR_FAIL(c, hipStreamWaitEvent(c->cs, K.ev_known, 0));
        kn = nw::OpsKnown{K.d_kstat.p, K.d_kmisc.p, K.d_kslots.p, K.d_kslots.p + 2 * nw::kOpsSlot, nw::kOpsSlot};
    }
    HIP_OR_FAIL(c, nw::launch_ops_compact(c->s->d_nops.p, c->s->d_slots.p, c->ops_slot, c->ops_stride, c->s->d_spill.p, c->n,
                                          c->s->d_lb.p, next_epoch(c), parity, c->d_ctl64.p + c->ctl_pass * nw::kOpsCtlAll,
                                          c->d_opsoff.p + c->out_off + base,
                                          c->s->d_staging.p, c->staging_cap, c->s->d_opsctl.p, cnt, c->cs, hctl, host,
                                          c->d_stats.p + c->out_off + base, c->known_on ? &kn : nullptr));
    tmark(c, "compact");
    return NW_OK;
}

// Page-locked host memory the device addresses with the same pointer (hipHostMalloc /
// hipHostRegister'd buffers, e.g. nw_host_alloc): kernels may store into it directly.
bool host_mapped(const void* p) {
    if (!p) return false;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost && at.devicePointer == p;
}

// NW_OUT_ROWS for the scope of a rows-only entry point (nw_align_batch, nw_align_multi)
struct RowsMode {
    nw_ctx* c;
    int saved;
    explicit RowsMode(nw_ctx* ctx) : c(ctx), saved(ctx->out_mode) { c->out_mode = NW_OUT_ROWS; }
    ~RowsMode() { c->out_mode = saved; }
};

int ops_events(nw_ctx* c, size_t chunks) {
    auto grow = [&](std::vector<hipEvent_t>& v, unsigned flags) -> hipError_t {
        while (v.size() < chunks) {
            hipEvent_t e = nullptr;
            hipError_t r = hipEventCreateWithFlags(&e, flags);
            if (r != hipSuccess) return r;
            v.push_back(e);
        }
        return hipSuccess;
    };
    HIP_OR_FAIL(c, grow(c->ev_in, hipEventDisableTiming));
    HIP_OR_FAIL(c, grow(c->ev_cs, hipEventDefault));
    HIP_OR_FAIL(c, grow(c->ev_ce, hipEventDefault));
    HIP_OR_FAIL(c, grow(c->ev_out, hipEventDisableTiming));
    HIP_OR_FAIL(c, grow(c->ev_bulk, hipEventDisableTiming));
    if ((int64_t)chunks > c->h_ctl_chunks) {
        if (c->h_ctl) (void)hipHostFree(c->h_ctl);
        c->h_ctl = nullptr;
        c->h_ctl_chunks = 0;
        HIP_OR_FAIL(c, hipHostMalloc((void**)&c->h_ctl, sizeof(int64_t) * nw::kOpsCtl * chunks, hipHostMallocDefault));
        c->h_ctl_chunks = (int64_t)chunks;
    }
    return NW_OK;
}

int ops_error(nw_ctx* c, int64_t err) {
    if (err & 4) return fail(c, NW_E_HIP, "a device prefix scan waited too long for its predecessor blocks");
    if (err & 2) return fail(c, NW_E_NOMEM, "ops spill area full: reads with more than %d traceback runs need more "
                                            "than the spill area (%lld MB)", c->ops_slot,
                             (long long)(c->spill_cap * 4 >> 20));
    if (err & 1) return fail(c, NW_E_NOMEM, "ops staging array full");
    return NW_OK;
}
}  // namespace

extern "C" {

int nw_batch_run_async(nw_ctx* c) {
    if (!c) return NW_E_INVALID;
    if (c->ref.empty() || !c->d_offsets.p) return fail(c, NW_E_STATE, "no batch uploaded");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipEventRecord(c->ev0, c->stream));
    int rc;
    c->call_done = false;
    c->phases = true;
    c->phases_recorded = c->phase_events;
    struct PhasesOff {
        nw_ctx* c;
        ~PhasesOff() { c->phases = false; }
    } phases_off{c};
    if (c->out_mode == NW_OUT_OPS) {
        if (!c->s->d_slots.p || c->s->d_nops.cap < (size_t)std::max<int64_t>(c->n, 1))
            return fail(c, NW_E_STATE, "batch uploaded before nw_batch_set_output(NW_OUT_OPS)");
        // the compaction's control block: zeroed by the band path's classify (the pass's first kernel;
        // a memset launch here cost two fill kernels, ~9 us, per pass), else by a memset
        if (c->use_diag && c->n > 0) {
            c->zero_ctl = c->d_ctl64.p;
        } else {
            HIP_OR_FAIL(c, hipMemsetAsync(c->d_ctl64.p, 0, nw::kOpsCtlAll * sizeof(int64_t), c->stream));
        }
        rc = launch_range_ops(c, 0);
        c->zero_ctl = nullptr;
    } else {
        rc = launch_range(c, 0);
    }
    if (rc) return rc;
    HIP_OR_FAIL(c, hipEventRecord(c->ev1, c->stream));
    c->ran = true;
    return NW_OK;
}

int nw_batch_sync(nw_ctx* c, float* kernel_ms) {
    if (!c) return NW_E_INVALID;
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    if (kernel_ms) {
        *kernel_ms = 0.0f;
        if (c->ran) HIP_OR_FAIL(c, hipEventElapsedTime(kernel_ms, c->ev0, c->ev1));
    }
    return NW_OK;
}

int nw_batch_download(nw_ctx* c, char* aln_out, int64_t stride, nw_stat* stats) {
    if (!c) return NW_E_INVALID;
    if (!c->ran) return fail(c, NW_E_STATE, "nothing has run");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    if (c->n == 0) return NW_OK;
    if (aln_out && c->out_mode == NW_OUT_OPS) return fail(c, NW_E_STATE, "ops output: use nw_batch_download_ops");
    if (c->use_diag) {   // the band path's single-pass scans report a cut-off look-back here
        int32_t fb[4] = {0, 0, 0, 0};
        HIP_OR_FAIL(c, hipMemcpy(fb, c->s->d_fallback_count.p, sizeof fb, hipMemcpyDeviceToHost));
        if (fb[3]) return ops_error(c, 4);
    }
    if (stats)
        HIP_OR_FAIL(c, hipMemcpy(stats, c->d_stats.p, sizeof(nw::Stat) * (size_t)c->n, hipMemcpyDeviceToHost));
    if (aln_out) {
        if (stride < c->stride) return fail(c, NW_E_INVALID, "stride %lld < required %lld", (long long)stride, (long long)c->stride);
        if (stride == c->stride) {
            HIP_OR_FAIL(c, hipMemcpy(aln_out, c->d_out.p, (size_t)c->n * 3 * c->stride, hipMemcpyDeviceToHost));
        } else {
            HIP_OR_FAIL(c, hipMemcpy2D(aln_out, (size_t)stride, c->d_out.p, (size_t)c->stride, (size_t)c->stride,
                                       (size_t)c->n * 3, hipMemcpyDeviceToHost));
        }
    }
    return NW_OK;
}

int64_t nw_batch_algo_bytes(nw_ctx* c) {
    if (!c || !c->ran) return -1;
    std::vector<nw::Stat> st((size_t)c->n);
    if (c->n && nw_batch_download(c, nullptr, 0, (nw_stat*)st.data()) != NW_OK) return -1;
    int64_t total = 0;
    for (int64_t r = 0; r < c->n; ++r)
        if (!(st[(size_t)r].flags & NW_FLAG_EMPTY)) total += c->read_lens[(size_t)r] + 3ll * st[(size_t)r].aln_len + 16;
    return total;
}

int64_t nw_batch_cells(const nw_ctx* c) { return c ? c->cells : -1; }

int nw_batch_kernel_times(nw_ctx* c, float* fill_ms, float* walk_ms, float* rest_ms) {
    if (!c) return NW_E_INVALID;
    if (!c->ran) return fail(c, NW_E_STATE, "nothing has run");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    float total = 0.0f, f = 0.0f, w = 0.0f;
    HIP_OR_FAIL(c, hipEventElapsedTime(&total, c->ev0, c->ev1));
    if (c->use_diag && c->n > 0 && !c->phases_recorded)
        return fail(c, NW_E_STATE, "the last run recorded no phase events (nw_batch_set_phase_events)");
    if (c->use_diag && c->n > 0) {
        HIP_OR_FAIL(c, hipEventElapsedTime(&f, c->ev0, c->ev_fill));
        HIP_OR_FAIL(c, hipEventElapsedTime(&w, c->ev_fill, c->ev_walk));
    } else {
        f = total;
    }
    if (fill_ms) *fill_ms = f;
    if (walk_ms) *walk_ms = w;
    if (rest_ms) *rest_ms = total - f - w;
    return NW_OK;
}

int nw_batch_device_output(nw_ctx* c, void** d_aln, int64_t* stride, void** d_stats) {
    if (!c) return NW_E_INVALID;
    if (!c->ran || c->n <= 0) return fail(c, NW_E_STATE, "no resident batch (run nw_batch_run_async first)");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    if (d_aln) *d_aln = c->d_out.p;
    if (stride) *stride = c->stride;
    if (d_stats) *d_stats = c->d_stats.p;
    return NW_OK;
}

int nw_batch_device_ops(nw_ctx* c, void** d_ops, void** d_ops_off, void** d_stats, void** d_reads, void** d_offsets,
                        int64_t* reads_bias, int64_t* max_cols) {
    if (!c) return NW_E_INVALID;
    if (!c->ran || c->n <= 0 || c->out_mode != NW_OUT_OPS)
        return fail(c, NW_E_STATE, "no resident ops-mode batch (nw_batch_set_output(NW_OUT_OPS), run first)");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    int64_t ctl[nw::kOpsCtl];
    HIP_OR_FAIL(c, hipMemcpy(ctl, c->d_ctl64.p, sizeof ctl, hipMemcpyDeviceToHost));
    int rc = ops_error(c, ctl[3]);
    if (rc) return rc;
    if (!c->bytes_full) {   // a packed batch: classify wrote the DP reads' bytes only; now every read's
        HIP_OR_FAIL(c, nw::launch_unpack((const uint32_t*)c->d_packed.p, c->batch_pos0 / 4, c->batch_base0,
                                         c->batch_base0 + c->batch_nbytes, c->d_exc_pos.p, c->d_exc_byte.p, 0,
                                         c->batch_n_exc, c->d_reads.p, c->reads_bias, c->stream));
        HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
        c->bytes_full = true;
    }
    if (d_ops) *d_ops = c->s->d_staging.p;   // one chunk: the call's runs from offset 0
    if (d_ops_off) *d_ops_off = c->d_opsoff.p;
    if (d_stats) *d_stats = c->d_stats.p;
    if (d_reads) *d_reads = c->d_reads.p;
    if (d_offsets) *d_offsets = c->d_offsets.p;
    if (reads_bias) *reads_bias = c->reads_bias;
    if (max_cols) *max_cols = c->stride;
    return NW_OK;
}

int nw_batch_geometry(const nw_ctx* c, int32_t* rows_per_lane, int32_t* waves_per_block, int32_t* grid,
                      int32_t* lds_bytes, int32_t* tb_mode) {
    if (!c) return NW_E_INVALID;
    const nw::LaunchCfg& k = c->use_diag ? c->diag_fill : c->cfg;
    if (rows_per_lane) *rows_per_lane = k.R;
    if (waves_per_block) *waves_per_block = k.wpb;
    if (grid) *grid = k.grid;
    if (lds_bytes) *lds_bytes = k.lds_bytes;
    if (tb_mode) *tb_mode = k.tb_mode;
    return NW_OK;
}

int64_t nw_batch_fallbacks(nw_ctx* c) {
    if (c && c->call_done) return c->call_counts[3];
    if (!c || !c->ran) return -1;
    (void)hipSetDevice(c->device);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    if (!c->use_diag) return 0;
    std::vector<int32_t> v(4);
    if (hipMemcpy(v.data(), c->s->d_fallback_count.p, v.size() * sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess)
        return -1;
    int64_t total = v[0];
    // a skipped second level (KernelArgs::redo_direct): its reads went to the exact kernel
    if (c->use_diag && c->diag16_fill.grid > 0 && c->redo_direct > 0 && v[2] <= c->redo_direct) total += v[2];
    return total;
}

int nw_align_batch(nw_ctx* c, const char* reads, const int64_t* offsets, int64_t n, char* aln_out,
                   int64_t stride, nw_stat* stats) {
    if (!c) return NW_E_INVALID;
    RowsMode rows_mode(c);
    int rc = nw_batch_upload(c, reads, offsets, n);
    if (rc) return rc;
    if ((rc = nw_batch_run_async(c))) return rc;
    if ((rc = nw_batch_sync(c, nullptr))) return rc;
    return nw_batch_download(c, aln_out, stride, stats);
}

// Pooled batches (CRISPRessoPooled.py:882-908 runs one CRISPResso
// process -- and one needle -- per amplicon): every read carries the index of
// its amplicon.  Reads are grouped by amplicon and uploaded once; each group's
// kernels are queued back to back on the context's stream (the profile upload
// of the next amplicon is ordered after them); one sync; outputs come back
// group by group and are scattered to the callers' read order.
int nw_align_multi(nw_ctx* c, const char* refs, const int64_t* ref_offsets, int32_t n_refs, const char* reads,
                   const int64_t* offsets, const int32_t* ref_of_read, int64_t n, char* aln_out, int64_t stride,
                   nw_stat* stats) {
    if (!c) return NW_E_INVALID;
    RowsMode rows_mode(c);
    if (n_refs <= 0 || !refs || !ref_offsets) return fail(c, NW_E_INVALID, "no amplicons");
    if (n < 0 || (n > 0 && (!reads || !offsets || !ref_of_read))) return fail(c, NW_E_INVALID, "bad batch");
    for (int32_t g = 0; g < n_refs; ++g) {
        const int64_t L = ref_offsets[g + 1] - ref_offsets[g];
        if (L <= 0 || L > kMaxRef) return fail(c, NW_E_UNSUPPORTED, "amplicon %d has length %lld", g, (long long)L);
    }
    (void)hipSetDevice(c->device);
    // group reads by amplicon (stable)
    std::vector<int64_t> first((size_t)n_refs + 1, 0);
    int32_t lb_all = 1;
    for (int64_t r = 0; r < n; ++r) {
        const int32_t g = ref_of_read[r];
        const int64_t len = offsets[r + 1] - offsets[r];
        if (g < 0 || g >= n_refs) return fail(c, NW_E_INVALID, "read %lld has amplicon index %d", (long long)r, g);
        if (len < 0 || len > (1 << 20)) return fail(c, NW_E_INVALID, "read %lld has length %lld", (long long)r, (long long)len);
        ++first[(size_t)g + 1];
        lb_all = std::max<int32_t>(lb_all, (int32_t)len);
    }
    for (int32_t g = 0; g < n_refs; ++g) first[(size_t)g + 1] += first[(size_t)g];
    std::vector<int64_t> order((size_t)n), fill(first.begin(), first.end() - 1);
    for (int64_t r = 0; r < n; ++r) order[(size_t)fill[(size_t)ref_of_read[r]]++] = r;
    int64_t stride_all = 16;
    for (int32_t g = 0; g < n_refs; ++g)
        if (first[(size_t)g + 1] > first[(size_t)g])
            stride_all = std::max(stride_all, stride_for((int)(ref_offsets[g + 1] - ref_offsets[g]), lb_all));
    if (aln_out && stride < stride_all)
        return fail(c, NW_E_INVALID, "stride %lld < required %lld", (long long)stride, (long long)stride_all);
    // packed reads in group order
    std::vector<int64_t> soff((size_t)n + 1, 0);
    for (int64_t s = 0; s < n; ++s) soff[(size_t)s + 1] = soff[(size_t)s] + (offsets[order[(size_t)s] + 1] - offsets[order[(size_t)s]]);
    std::vector<char> sreads((size_t)soff[(size_t)n]);
    for (int64_t s = 0; s < n; ++s) {
        const int64_t r = order[(size_t)s];
        std::memcpy(sreads.data() + soff[(size_t)s], reads + offsets[r], (size_t)(offsets[r + 1] - offsets[r]));
    }
    c->resident_ok = false;
    HIP_OR_FAIL(c, c->d_reads.reserve(sreads.size() + 512));
    HIP_OR_FAIL(c, c->d_offsets.reserve((size_t)n + 1));
    HIP_OR_FAIL(c, c->d_out.reserve((size_t)std::max<int64_t>(n, 1) * 3 * stride_all));
    HIP_OR_FAIL(c, c->d_stats.reserve((size_t)std::max<int64_t>(n, 1)));
    HIP_OR_FAIL(c, c->s->d_fallback.reserve((size_t)std::max<int64_t>(n, 1)));
    HIP_OR_FAIL(c, c->s->d_fallback2.reserve((size_t)std::max<int64_t>(n, 1)));   // indexed like d_fallback (+ group base)
    if (!sreads.empty())
        HIP_OR_FAIL(c, hipMemcpyAsync(c->d_reads.p, sreads.data(), sreads.size(), hipMemcpyHostToDevice, c->stream));
    HIP_OR_FAIL(c, hipMemcpyAsync(c->d_offsets.p, soff.data(), sizeof(int64_t) * soff.size(), hipMemcpyHostToDevice, c->stream));
    // every amplicon's tables uploaded once (one arena); then one kernel group per amplicon,
    // queued back to back on the stream (configure() may grow buffers between groups)
    std::vector<std::string> amps((size_t)n_refs);
    for (int32_t g = 0; g < n_refs; ++g) amps[(size_t)g].assign(refs + ref_offsets[g], refs + ref_offsets[g + 1]);
    std::vector<Profile> profs;
    {
        int rc = upload_shared(c);
        if (!rc) rc = upload_profiles(c, amps, &profs);
        if (rc) return rc;
    }
    for (int32_t g = 0; g < n_refs; ++g) {
        const int64_t lo = first[(size_t)g], hi = first[(size_t)g + 1];
        if (hi == lo) continue;
        c->ref = amps[(size_t)g];
        c->cur = profs[(size_t)g];
        int rc = NW_OK;
        int32_t lb = 1;
        int64_t cells = 0;
        for (int64_t s = lo; s < hi; ++s) {
            const int64_t len = soff[(size_t)s + 1] - soff[(size_t)s];
            lb = std::max<int32_t>(lb, (int32_t)len);
            cells += (int64_t)c->ref.size() * len;
        }
        c->n = hi - lo;
        c->lb_max = lb;
        c->cells = cells;
        c->stride = stride_all;
        if ((rc = configure(c))) return rc;
        if ((rc = launch_range(c, lo))) return rc;
    }
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    // back to the callers' order
    std::vector<nw::Stat> st((size_t)n);
    if (n) HIP_OR_FAIL(c, hipMemcpy(st.data(), c->d_stats.p, sizeof(nw::Stat) * (size_t)n, hipMemcpyDeviceToHost));
    if (stats)
        for (int64_t s = 0; s < n; ++s) std::memcpy(&stats[order[(size_t)s]], &st[(size_t)s], sizeof(nw::Stat));
    if (aln_out) {
        std::vector<char> rows;
        for (int32_t g = 0; g < n_refs; ++g) {
            const int64_t lo = first[(size_t)g], hi = first[(size_t)g + 1];
            if (hi == lo) continue;
            rows.resize((size_t)(hi - lo) * 3 * stride_all);
            HIP_OR_FAIL(c, hipMemcpy(rows.data(), c->d_out.p + lo * 3 * stride_all, rows.size(), hipMemcpyDeviceToHost));
            for (int64_t s = lo; s < hi; ++s)
                for (int k = 0; k < 3; ++k)
                    std::memcpy(aln_out + (order[(size_t)s] * 3 + k) * stride, rows.data() + ((s - lo) * 3 + k) * stride_all,
                                (size_t)stride_all);
        }
    }
    c->n = 0;          // the per-batch getters describe nw_batch_upload batches only
    c->ran = false;
    c->ref.clear();    // the arena holds every amplicon: nw_set_reference before single-amplicon calls
    c->cur = Profile{};
    c->call_done = false;
    return NW_OK;
}

int64_t nw_required_stride_multi(const int64_t* ref_offsets, int32_t n_refs, int32_t max_read_len) {
    if (!ref_offsets || n_refs <= 0) return 0;
    int64_t st = 16;
    for (int32_t g = 0; g < n_refs; ++g)
        st = std::max(st, stride_for((int)(ref_offsets[g + 1] - ref_offsets[g]), std::max(max_read_len, 1)));
    return st;
}

int nw_batch_set_output(nw_ctx* c, int mode) {
    if (!c) return NW_E_INVALID;
    if (mode != NW_OUT_ROWS && mode != NW_OUT_OPS) return fail(c, NW_E_INVALID, "output mode %d", mode);
    c->out_mode = mode;
    c->ran = false;
    c->call_done = false;
    return NW_OK;
}

int nw_batch_download_ops(nw_ctx* c, uint32_t* ops_out, int64_t ops_cap, int64_t* ops_off, nw_stat* stats) {
    if (!c) return NW_E_INVALID;
    if (!c->ran || c->out_mode != NW_OUT_OPS) return fail(c, NW_E_STATE, "no ops-mode run (nw_batch_set_output)");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    int64_t ctl[nw::kOpsCtl];
    HIP_OR_FAIL(c, hipMemcpy(ctl, c->d_ctl64.p, sizeof ctl, hipMemcpyDeviceToHost));
    int rc = ops_error(c, ctl[3]);
    if (rc) return rc;
    if (c->n > 0) {
        if (stats) HIP_OR_FAIL(c, hipMemcpy(stats, c->d_stats.p, sizeof(nw::Stat) * (size_t)c->n, hipMemcpyDeviceToHost));
        if (ops_off) HIP_OR_FAIL(c, hipMemcpy(ops_off, c->d_opsoff.p, sizeof(int64_t) * (size_t)c->n, hipMemcpyDeviceToHost));
    }
    if (ops_off) ops_off[c->n] = ctl[2];
    if (ctl[2] > ops_cap)
        return fail(c, NW_E_CAPACITY, "ops_cap %lld < %lld runs", (long long)ops_cap, (long long)ctl[2]);
    if (ctl[2] > 0 && ops_out)
        HIP_OR_FAIL(c, hipMemcpy(ops_out, c->s->d_staging.p, sizeof(uint32_t) * (size_t)ctl[2], hipMemcpyDeviceToHost));
    return NW_OK;
}

// The call-level path (host batch in -> per-read records in host
// memory).  Chunks of reads flow through three streams: every chunk's reads and
// offsets are queued on s_in up front; chunk k's kernels + compaction wait for its
// upload on the compute stream; its records and offsets go back on s_out as soon as
// they exist, its runs once the host has read the chunk's run total (the host waits
// for chunk k - 1 while chunk k computes).  Compute of chunk k + 2 reuses chunk k's
// staging array after its copy.  Host buffers should be pinned (nw_host_alloc /
// nw_host_register) for the copies to run asynchronously at PCIe rate.
}  // extern "C"

namespace {

// CRISPR_NW_HOST_TIMING=1: where a pipelined call's host time goes (stderr; diagnostics)
struct HostTimer {
    bool on = false;
    const char* what;
    double t[8] = {0, 0, 0, 0, 0, 0, 0, 0};   // ops_call: scan, configure, setup, uploads, launch, wait, sync
    std::chrono::steady_clock::time_point t0, last;
    explicit HostTimer(const char* w) : what(w) {
        const char* e = std::getenv("CRISPR_NW_HOST_TIMING");
        on = e && std::strcmp(e, "1") == 0;
        t0 = last = std::chrono::steady_clock::now();
    }
    void lap(int k) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        t[k] += std::chrono::duration<double, std::milli>(now - last).count();
        last = now;
    }
    ~HostTimer() {
        if (!on) return;
        t[7] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        std::fprintf(stderr, "nw host ms (%s): %.2f %.2f %.2f %.2f %.2f %.2f %.2f total %.2f\n", what, t[0], t[1], t[2],
                     t[3], t[4], t[5], t[6], t[7]);
    }
};

// What configure() decides for one amplicon (launch configurations, path choice,
// geometry): a pooled call configures every group once up front and restores these
// per chunk instead of re-running configure (its occupancy queries are host API calls).
struct CfgState {
    nw::LaunchCfg cfg, diag_fill, diag_walk, diag16_fill, diag16_walk, wide_fill, wide_walk;
    int64_t wide_pairs, wide_stride;
    int wide_words, wide_lb_cap;
    bool use_diag, exact_tb_lds, exact_full;
    int exact_grid, exact_lds, diag_words, diag_lb_cap;
    int64_t exact_slab, diag16_pass_pairs, diag16_stride, diag_pass_pairs, diag_stride, stride;
};
CfgState save_cfg(const nw_ctx* c) {
    return CfgState{c->cfg, c->diag_fill, c->diag_walk, c->diag16_fill, c->diag16_walk, c->wide_fill, c->wide_walk,
                    c->wide_pairs, c->wide_stride, c->wide_words, c->wide_lb_cap, c->use_diag, c->exact_tb_lds,
                    c->exact_full, c->exact_grid, c->exact_lds, c->diag_words, c->diag_lb_cap,
                    c->exact_slab, c->diag16_pass_pairs, c->diag16_stride, c->diag_pass_pairs, c->diag_stride,
                    c->stride};
}
void load_cfg(nw_ctx* c, const CfgState& st) {
    c->cfg = st.cfg; c->diag_fill = st.diag_fill; c->diag_walk = st.diag_walk; c->diag16_fill = st.diag16_fill;
    c->diag16_walk = st.diag16_walk; c->use_diag = st.use_diag; c->exact_tb_lds = st.exact_tb_lds;
    c->exact_full = st.exact_full; c->exact_grid = st.exact_grid; c->exact_lds = st.exact_lds;
    c->diag_words = st.diag_words; c->diag_lb_cap = st.diag_lb_cap;
    c->exact_slab = st.exact_slab; c->diag16_pass_pairs = st.diag16_pass_pairs; c->diag16_stride = st.diag16_stride;
    c->diag_pass_pairs = st.diag_pass_pairs; c->diag_stride = st.diag_stride; c->stride = st.stride;
    c->wide_fill = st.wide_fill; c->wide_walk = st.wide_walk; c->wide_pairs = st.wide_pairs;
    c->wide_stride = st.wide_stride; c->wide_words = st.wide_words; c->wide_lb_cap = st.wide_lb_cap;
}

// 2-bit packed batch (nw_align_ops_packed): bases by batch position, exceptions ascending.
struct PackedInput {
    const uint8_t* packed;
    const int64_t* exc_pos;
    const uint8_t* exc_byte;
    int64_t n_exc;
    const uint16_t* lens = nullptr;   // the reads' lengths (nw_align_ops_packed_lens): they cross instead of the offsets
};

// Amplicon groups of a pooled call: reads [first[g], first[g + 1]) align against
// refs[g] (tables profs[g] in the arena).
struct Groups {
    const std::vector<std::string>* refs;
    const std::vector<Profile>* profs;
    const std::vector<int64_t>* first;
};

// A dual call (nw_align_dual_ops_packed_lens, CORE:1808-1828): every read against refs[0] (pass 0:
// the caller's stats / ops_off / ops_out) and refs[1] (pass 1: these outputs; null ops_out2: records
// only), the two passes' chunks interleaved -- pass 1's chunk of a read range runs as soon as that
// range is uploaded, on the time the upload-bound pass 0 leaves the GPU idle.
struct Dual {
    uint32_t* ops_out2;
    int64_t ops_cap2;
    int64_t* ops_off2;
    nw_stat* stats2;
};

// Known copies (nw_ctx::resident_ref): the resident batch was aligned against amplicon A and is
// now aligned against H (the HDR pass, CORE:1808-1828): reads equal to A all have A's alignment
// against H.  A goes through the exact kernel once, as a one-read batch with its own buffers, on
// the upload stream (idle in a resident pass) while the chunks start; classify flags A's copies
// (KernelArgs::known2) and every chunk's compaction waits for the alignment and gives it to them.
// Off unless both sequences are A C G T, of one length <= 256 (classify's lane-per-read compare)
// and at most the batch's longest read (the exact kernel's LDS sizing).
int known_prepare(nw_ctx* c, const std::string& A, hipStream_t ks, int set = 0) {
    auto& K = c->kset[set];
    K.on = false;
    const int La = (int)c->ref.size();
    if ((int)A.size() != La || La > 256 || La > c->lb_max || A == c->ref || !c->cur.amp_acgt || !c->cur.amp2 ||
        c->cfg.R <= 0 || c->end_weight)
        return NW_OK;
    for (char ch : A) {
        const char u = (char)(ch & 0xDF);
        if (u != 'A' && u != 'C' && u != 'G' && u != 'T') return NW_OK;
    }
    std::vector<uint32_t> w2((size_t)(La + 15) / 16 + 2, 0u);
    for (int p = 0; p < La; ++p) w2[(size_t)p / 16] |= (uint32_t)(((unsigned char)A[p] >> 1) & 3u) << (2 * (p % 16));
    const int64_t tbw = c->cfg.tb_mode == nw::TB_GLOBAL_FULL ? nw::tb_bytes_per_wave(c->cfg.R, c->lb_max) : 0;
    HIP_OR_FAIL(c, K.d_kbytes.reserve((size_t)La + 64));
    HIP_OR_FAIL(c, K.d_koff.reserve(2));
    HIP_OR_FAIL(c, K.d_k2.reserve(w2.size()));
    HIP_OR_FAIL(c, K.d_kslots.reserve(2 * nw::kOpsSlot + 4096));   // column-major + row-major slot, spill
    HIP_OR_FAIL(c, K.d_kstat.reserve(1));
    HIP_OR_FAIL(c, K.d_kmisc.reserve(16));
    HIP_OR_FAIL(c, K.d_kfb.reserve(1));
    HIP_OR_FAIL(c, K.d_ktb.reserve((size_t)std::max<int64_t>(tbw * c->cfg.wpb, 16)));
    if (!K.ev_known) HIP_OR_FAIL(c, hipEventCreateWithFlags(&K.ev_known, hipEventDisableTiming));
    const int64_t off[2] = {0, La};
    HIP_OR_FAIL(c, hipMemcpyAsync(K.d_kbytes.p, A.data(), (size_t)La, hipMemcpyHostToDevice, ks));
    HIP_OR_FAIL(c, hipMemcpyAsync(K.d_koff.p, off, sizeof off, hipMemcpyHostToDevice, ks));
    HIP_OR_FAIL(c, hipMemcpyAsync(K.d_k2.p, w2.data(), 4 * w2.size(), hipMemcpyHostToDevice, ks));
    HIP_OR_FAIL(c, hipMemsetAsync(K.d_kmisc.p, 0, 16 * sizeof(int32_t), ks));
    nw::KernelArgs ka{};
    ka.reads = K.d_kbytes.p;
    ka.offsets = K.d_koff.p;
    ka.n = 1;
    ka.prof = c->cur.prof;
    ka.lut = c->d_lut.p;
    ka.amp = c->cur.amp;
    ka.La = La;
    ka.gap_open = c->gap_open;
    ka.gap_extend = c->gap_extend;
    ka.Lb_max = c->lb_max;
    ka.stats = K.d_kstat.p;
    ka.tb_global = K.d_ktb.p;
    ka.tb_wave_bytes = tbw;
    ka.fallback_list = K.d_kfb.p;
    ka.fallback_count = K.d_kmisc.p + 8;
    ka.ops = K.d_kslots.p;
    ka.ops_slot = nw::kOpsSlot;
    ka.ops_stride = 1;
    ka.nops = K.d_kmisc.p;
    ka.spill = K.d_kslots.p + 2 * nw::kOpsSlot;
    ka.spill_cap = 4096;
    ka.ops_ctl = K.d_kmisc.p + 1;
    nw::LaunchCfg one = c->cfg;
    one.grid = 1;
    HIP_OR_FAIL(c, nw::launch(ka, one, ks));
    HIP_OR_FAIL(c, hipEventRecord(K.ev_known, ks));
    K.on = true;
    return NW_OK;
}

// nw_align_ops (upload = true), nw_align_ops_resident (the batch the last call
// uploaded, still in HBM: no upload) and nw_align_multi_ops (groups: chunks never
// straddle two amplicons; each chunk's kernels use its amplicon's tables).
int ops_call(nw_ctx* c, const char* reads, const int64_t* offsets, int64_t n, uint32_t* ops_out, int64_t ops_cap,
             int64_t* ops_off, nw_stat* stats, bool upload, const Groups* groups = nullptr,
             const PackedInput* pk = nullptr, const Dual* dual = nullptr) {
    if (!c) return NW_E_INVALID;
    if (dual && (!groups || groups->refs->size() != 2 || !upload || !pk || !dual->stats2 || !dual->ops_off2))
        return fail(c, NW_E_INVALID, "bad dual call");
    HostTimer ht("scan configure setup uploads launch wait sync");
    if (!groups && c->ref.empty()) return fail(c, NW_E_STATE, "nw_set_reference must come first");
    if (n < 0 || (n > 0 && (!offsets || (upload && !reads && !(pk && pk->packed)) || !stats)) || !ops_off)
        return fail(c, NW_E_INVALID, "bad batch");
    if (pk && pk->n_exc > 0 && (!pk->exc_pos || !pk->exc_byte)) return fail(c, NW_E_INVALID, "bad exception list");
    if (!upload && !(c->resident_ok && c->resident_n == n && (n == 0 || (c->resident_lo == offsets[0] &&
                                                                          c->resident_hi == offsets[n]))))
        return fail(c, NW_E_STATE, "no resident batch of these %lld reads (nw_align_ops uploads one)", (long long)n);
    if (upload) c->resident_ok = false;
    (void)hipSetDevice(c->device);
    int64_t chunk = 262144;
    if (const char* e = std::getenv("CRISPR_NW_CHUNK")) chunk = std::max(1ll, std::atoll(e));
    chunk = std::max<int64_t>(1, std::min<int64_t>(chunk, n));
    // chunks [lo, hi) of one amplicon group each; a dual call's pass-1 chunk reads the bytes its
    // pass-0 twin (chunk `up`) uploaded
    struct Chunk { int64_t lo, hi; int g; int pass; int64_t up; };
    std::vector<Chunk> chunks;
    const int ngroups = groups ? (int)groups->refs->size() : 1;
    // sizes ramp up and down at both ends of the call (chunk / 4, chunk / 2, ...): the
    // first chunk's upload and the last chunk's records are the pipeline's serial head
    // and tail; every chunk in between is a full chunk
    // (8:4:2 ramps and other chunk sizes measured no faster)
    auto sizes = [&](int64_t len) {
        std::vector<int64_t> v;
        if (len <= chunk) {
            v.push_back(len);
            return v;
        }
        std::vector<int64_t> head, tail;
        int64_t left = len;
        for (int64_t part : {chunk / 4, chunk / 2}) {   // ramp parts in pairs (one at each end)
            if (part >= 1024 && left > 2 * (part + chunk)) {
                head.push_back(part);
                tail.push_back(part);
                left -= 2 * part;
            }
        }
        for (int64_t x : head) v.push_back(x);
        const int64_t mid = (left + chunk - 1) / chunk;
        for (int64_t q = 0; q < mid; ++q) v.push_back(left / mid + (q < left % mid ? 1 : 0));
        for (auto it = tail.rbegin(); it != tail.rend(); ++it) v.push_back(*it);
        return v;
    };
    if (dual) {
        int64_t lo = 0;
        for (int64_t len : sizes(n)) {
            if (len <= 0) continue;
            const int64_t k0 = (int64_t)chunks.size();
            chunks.push_back({lo, lo + len, 0, 0, k0});
            chunks.push_back({lo, lo + len, 1, 1, k0});
            lo += len;
        }
    } else {
        for (int g = 0; g < ngroups; ++g) {
            const int64_t g0 = groups ? (*groups->first)[(size_t)g] : 0, g1 = groups ? (*groups->first)[(size_t)g + 1] : n;
            int64_t lo = g0;
            for (int64_t len : sizes(g1 - g0)) {
                if (len <= 0) continue;
                chunks.push_back({lo, lo + len, g, 0, (int64_t)chunks.size()});
                lo += len;
            }
        }
    }
    // chunk k's predecessor of its own pass, the newest chunk of its pass the host has read back
    // lag chunks behind it, and its index within its pass (a dual call's passes alternate)
    auto prev_same = [&](int64_t j) { return dual ? j - 2 : j - 1; };
    auto newest_same = [&](int64_t k, int64_t back) {
        int64_t j = k - back;
        if (dual && j >= 0 && chunks[(size_t)j].pass != chunks[(size_t)k].pass) --j;
        return j;
    };
    auto in_pass = [&](int64_t k) { return dual ? k >> 1 : k; };
    const int mode_before = c->out_mode;
    const int64_t base0 = n ? offsets[0] : 0;
    const int64_t nbytes = n ? offsets[n] - base0 : 0;
    const int64_t nchunks = (int64_t)chunks.size();
    auto restore = [&](int code) {
        c->seed_on = false;
        c->seed_chunk = false;
        c->seed_pairs = 0;
        c->split_to = nullptr;
        c->skip16 = false;
        c->exact_small = false;
        c->trace_on = false;
        c->known_on = false;
        c->lane_call = false;
        c->kcur = 0;
        c->out_off = 0;
        c->ctl_pass = 0;
        c->pkc = nw::KernelArgs{};
        c->out_mode = mode_before;
        c->n = 0;
        c->s = &c->sc[0];
        c->cs = c->stream;
        return code;
    };
    int rc = NW_OK;
    // the chunks' edges must be in order before anything is copied (the scan below checks
    // every read, after the uploads are queued: the copy engine starts streaming at once)
    for (const Chunk& ch : chunks)
        if (offsets[ch.lo] > offsets[ch.hi] || offsets[ch.lo] < base0 || offsets[ch.hi] > offsets[n])
            return fail(c, NW_E_INVALID, "offsets out of order at read %lld", (long long)ch.lo);
    // packed input: the device copy of the packed stream starts at byte P0 (4-aligned: one
    // dword = 16 bases), the unpacked bytes at batch position base0 & ~15 (16-B stores)
    const int64_t P0 = (base0 / 16) * 4;
    const int64_t pk_hi = n ? (offsets[n] + 3) / 4 : 0;   // end of the caller's packed bytes
    if (pk && upload &&
        (c->d_packed.reserve((size_t)std::max<int64_t>(pk_hi - P0, 0) + 64) != hipSuccess ||
         c->d_exc_pos.reserve((size_t)std::max<int64_t>(pk->n_exc, 1)) != hipSuccess ||
         c->d_exc_byte.reserve((size_t)std::max<int64_t>(pk->n_exc, 1)) != hipSuccess))
        return restore(fail(c, NW_E_NOMEM, "device allocation failed for the packed batch"));
    if (c->d_reads.reserve((size_t)nbytes + 512 + 16) != hipSuccess || c->d_offsets.reserve((size_t)n + 1) != hipSuccess ||
        c->d_stats.reserve((size_t)std::max<int64_t>(dual ? 2 * n + 2 : n, 1)) != hipSuccess)
        return restore(fail(c, NW_E_NOMEM, "device allocation failed for %lld reads", (long long)n));
    if ((rc = ops_events(c, (size_t)std::max<int64_t>(nchunks, 1)))) return restore(rc);
    ht.lap(2);
    if (upload) c->reads_bias = pk ? (base0 & ~(int64_t)15) : base0;
    // every upload queued up front: the copy engine streams the batch while chunks compute
    HIP_OR_FAIL(c, hipEventRecord(c->ev_h0, c->s_in));
    int64_t h2d_bytes = 0;
    if (pk && upload && pk->n_exc > 0) {
        HIP_OR_FAIL(c, hipMemcpyAsync(c->d_exc_pos.p, pk->exc_pos, sizeof(int64_t) * (size_t)pk->n_exc,
                                      hipMemcpyHostToDevice, c->s_in));
        HIP_OR_FAIL(c, hipMemcpyAsync(c->d_exc_byte.p, pk->exc_byte, (size_t)pk->n_exc, hipMemcpyHostToDevice, c->s_in));
        h2d_bytes += 9 * pk->n_exc;
    }
    // Packed input with the reads' lengths (nw_align_ops_packed_lens): per read its uint16
    // length crosses PCIe instead of its int64 offset (plus every kLenGroup-th offset, once):
    // 2 B instead of 8, 70.5 -> 64.5 MB per 1M C2 reads.  The call is PCIe-bound at the
    // margin (8 MB more upload measured +0.15 ms).  Each chunk's unpack launch rebuilds its
    // offsets (nw::LenSeg); the scan below checks the lengths against the group offsets
    // before any kernel runs.
    const bool lens_on = pk && pk->lens && upload && n > 0;
    const int64_t ngroups_len = lens_on ? n / nw::kLenGroup + 1 : 0;
    int64_t mx = 1, mn = 0;
    int64_t n_short = 0;   // reads the 16-diagonal band cannot hold (Lb <= La - 16): the seeded band's
    const int64_t short_la = ngroups == 1 ? (int64_t)c->ref.size() : 0;
    if (lens_on) {
        // the group bases and chunk 0's lengths in one copy (the device layout is [bases][lengths])
        const int64_t n0 = nchunks > 0 ? chunks[0].hi - chunks[0].lo : 0;
        const int64_t need = 8 * ngroups_len + 2 * n0;
        if (need > c->h_lens_cap) {
            if (c->h_lens) (void)hipHostFree(c->h_lens);
            c->h_lens = nullptr;
            c->h_lens_cap = 0;
            HIP_OR_FAIL(c, hipHostMalloc((void**)&c->h_lens, (size_t)need, hipHostMallocDefault));
            c->h_lens_cap = need;
        }
        if (c->d_lens.reserve((size_t)(8 * ngroups_len + 2 * n + 64)) != hipSuccess)
            return restore(fail(c, NW_E_NOMEM, "device allocation failed for %lld reads", (long long)n));
        int64_t* gb = (int64_t*)c->h_lens;
        for (int64_t g = 0; g < ngroups_len; ++g) gb[g] = offsets[g * nw::kLenGroup];
        std::memcpy(c->h_lens + 8 * ngroups_len, pk->lens + chunks[0].lo, 2 * (size_t)n0);
        HIP_OR_FAIL(c, hipMemcpyAsync(c->d_lens.p, c->h_lens, (size_t)need, hipMemcpyHostToDevice, c->s_in));
        h2d_bytes += need;
    }
    nw_host::Pool& pool = nw_host::Pool::get();
    for (int64_t k = 0; upload && k < nchunks; ++k) {
        if (chunks[(size_t)k].pass) continue;   // its twin's upload holds its reads
        const int64_t lo = chunks[(size_t)k].lo, hi = chunks[(size_t)k].hi;
        const int64_t b0 = offsets[lo], b1 = offsets[hi];
        // chunk 0's lengths went with the group bases; every later chunk's in one copy queued
        // ahead of chunk 1's bases: fewer copies, fewer gaps on the engine (C4 16.9 -> 16.4 ms,
        // C5 17.2 -> 17.0 ms against one lengths copy per chunk)
        if (lens_on && k == (dual ? 2 : 1)) {
            HIP_OR_FAIL(c, hipMemcpyAsync(c->d_lens.p + 8 * ngroups_len + 2 * lo, pk->lens + lo, 2 * (size_t)(n - lo),
                                          hipMemcpyHostToDevice, c->s_in));
            h2d_bytes += 2 * (n - lo);
        }
        if (pk) {
            // the chunk's packed dwords (the caller's bytes only; edge bases are masked)
            const int64_t q0 = std::max((b0 / 16) * 4, base0 / 4), q1 = std::min((b1 + 15) / 16 * 4, pk_hi);
            if (b1 > b0 && q1 > q0) {
                HIP_OR_FAIL(c, hipMemcpyAsync(c->d_packed.p + (q0 - P0), pk->packed + q0, (size_t)(q1 - q0),
                                              hipMemcpyHostToDevice, c->s_in));
                h2d_bytes += q1 - q0;
            }
        } else if (b1 > b0) {
            HIP_OR_FAIL(c, hipMemcpyAsync(c->d_reads.p + (b0 - base0), reads + b0, (size_t)(b1 - b0), hipMemcpyHostToDevice,
                                          c->s_in));
            h2d_bytes += b1 - b0;
        }
        if (!lens_on) {
            HIP_OR_FAIL(c, hipMemcpyAsync(c->d_offsets.p + lo, offsets + lo, sizeof(int64_t) * (size_t)(hi - lo + 1),
                                          hipMemcpyHostToDevice, c->s_in));
            h2d_bytes += (int64_t)sizeof(int64_t) * (hi - lo + 1);
        }
        HIP_OR_FAIL(c, hipEventRecord(c->ev_in[(size_t)k], c->s_in));
    }
    if (upload) HIP_OR_FAIL(c, hipEventRecord(c->ev_h1, c->s_in));
    ht.lap(3);
    // lengths given: the longest read, and every length must equal its offsets' difference
    // (the device rebuilds the offsets from the lengths and the group bases, the host expands
    // the rows from the offsets: a mismatch would make them refer to different bytes)
    if (lens_on) {
        const int parts = (int)std::min<int64_t>(pool.threads(), std::max<int64_t>(1, n >> 16));
        std::vector<int64_t> pmx((size_t)parts, 1), pbad((size_t)parts, -1), psh((size_t)parts, 0);
        pool.run(parts, [&](int q) {
            int64_t g0, g1;
            nw_host::Pool::range(ngroups_len, parts, q, &g0, &g1);
            unsigned a = 1;
            int64_t sh = 0;
            for (int64_t g = g0; g < g1 && pbad[(size_t)q] < 0; ++g) {
                const int64_t r0 = g * nw::kLenGroup, r1 = std::min(n, r0 + nw::kLenGroup);
                int64_t diff = 0;
                for (int64_t r = r0; r < r1; ++r) {
                    const unsigned l = pk->lens[r];
                    a = l > a ? l : a;
                    sh += (int64_t)l + 16 <= short_la;
                    diff |= (int64_t)l ^ (offsets[r + 1] - offsets[r]);
                }
                if (diff) pbad[(size_t)q] = g;
            }
            pmx[(size_t)q] = a;
            psh[(size_t)q] = sh;
        });
        for (int q = 0; q < parts; ++q) {
            mx = std::max(mx, pmx[(size_t)q]);
            n_short += psh[(size_t)q];
            if (pbad[(size_t)q] >= 0) {
                (void)hipStreamSynchronize(c->s_in);   // the queued uploads read the caller's arrays
                return restore(fail(c, NW_E_INVALID, "lens differ from the offsets in reads %lld ..",
                                    (long long)(pbad[(size_t)q] * nw::kLenGroup)));
            }
        }
    }
    // longest / shortest read: a vectorisable pass, split over the host pool for large
    // batches (memory-bound; the exact read is found only on error)
    if (!lens_on) {
        const int parts = (int)std::min<int64_t>(pool.threads(), std::max<int64_t>(1, n >> 15));
        std::vector<int64_t> pmx((size_t)parts, 1), pmn((size_t)parts, 0), psh((size_t)parts, 0);
        pool.run(parts, [&](int q) {
            int64_t lo, hi, a = 1, b = 0, sh = 0;
            nw_host::Pool::range(n, parts, q, &lo, &hi);
            for (int64_t r = lo; r < hi; ++r) {
                const int64_t len = offsets[r + 1] - offsets[r];
                a = len > a ? len : a;
                b = len < b ? len : b;
                sh += len + 16 <= short_la;
            }
            pmx[(size_t)q] = a;
            pmn[(size_t)q] = b;
            psh[(size_t)q] = sh;
        });
        for (int q = 0; q < parts; ++q) {
            mx = std::max(mx, pmx[(size_t)q]);
            mn = std::min(mn, pmn[(size_t)q]);
            n_short += psh[(size_t)q];
        }
    }
    if (mn < 0 || mx > (1 << 20))
        for (int64_t r = 0; r < n; ++r) {
            const int64_t len = offsets[r + 1] - offsets[r];
            if (len < 0 || len > (1 << 20))
            {
                (void)hipStreamSynchronize(c->s_in);   // the queued uploads read the caller's arrays
                return restore(fail(c, NW_E_INVALID, "read %lld has length %lld", (long long)r, (long long)len));
            }
        }
    const int32_t lb_max = (int32_t)mx;
    // the seeded band: a one-amplicon call whose classify decodes a packed batch
    // (an upload, or the resident batch of one), with reads the 16-diagonal band cannot hold; its
    // sort keys must fit the segment sort (11 key bits, LDS)
    {
        const int La = (int)c->ref.size();
        const int keys = La / 2 + 2, cap = La + nw::kBandDiags - 1;
        // (a few such reads -- C2's long deletions -- the 32-diagonal level holds: not worth the keys)
        c->seed_on = ngroups == 1 && n_short > 0 && 64 * n_short >= n && (pk != nullptr || (!upload && c->resident_packed)) &&
                     !c->end_weight && La <= 1024 && cap + 3 + keys <= 2048 &&
                     4 * 17 * (cap + keys + 3) + 128 <= 64 * 1024;   // segsort_lds_bytes (default LDS limit)
        c->seed_keys = c->seed_on ? keys : 0;
        const char* e2 = std::getenv("CRISPR_NW_SEED32");   // "0": the seeded list straight to the wide level (tests, A/Bs)
        c->seed_l2 = !(e2 && std::atoi(e2) == 0);
        c->seed_pairs = c->seed_on ? std::min<int64_t>(chunk, n_short) / 2 + 1 : 0;
    }
    ht.lap(0);
    c->out_mode = NW_OUT_OPS;
    c->ran = false;
    c->call_done = false;
    c->lb_max = lb_max;
    c->cells = 0;
    // launch configuration of a chunk: configure() for its amplicon group once (grids sized
    // for a full chunk also serve a shorter last chunk: the kernels clamp to the counts)
    int configured = -1;
    std::vector<CfgState> gcfg;        // per group, from the dry pass (pooled calls)
    std::vector<char> have_cfg((size_t)ngroups, 0);
    if (groups) gcfg.resize((size_t)ngroups);
    auto use_group = [&](int g, int64_t reads_in_chunk) {
        if (g == configured) {
            c->n = reads_in_chunk;
            return (int)NW_OK;
        }
        if (groups) {
            c->ref = (*groups->refs)[(size_t)g];
            c->cur = (*groups->profs)[(size_t)g];
            if (have_cfg[(size_t)g]) {   // restored, not re-derived (buffers were sized by the dry pass)
                load_cfg(c, gcfg[(size_t)g]);
                c->n = reads_in_chunk;
                configured = g;
                return (int)NW_OK;
            }
        }
        c->stride = stride_for((int)c->ref.size(), lb_max);
        c->n = std::max(reads_in_chunk, std::min<int64_t>(chunk, n));
        const int r = configure(c);
        c->n = reads_in_chunk;
        configured = r ? -1 : g;
        return r;
    };
    // configure every group once up front: the buffers reach their largest size before
    // anything is queued (no allocation inside the pipeline)
    // (A resident pass -- the C3 HDR pass -- in 524288- / 1048576-read chunks measured 8.95 / 10.77
    // vs 5.85 ms per C3 step: the wide level's region per chunk overflows to the exact kernel and the
    // last chunk's records go over PCIe unoverlapped; without the tail stream 5.78 vs 5.70.)
    // two sets overlap a chunk's tail with the next chunk's bulk; a third measured slower
    // (328M vs 306M reads/s at 262144-read chunks, scripts/gpu_sets_sweep.sh)
    const bool several = (n + chunk - 1) / std::max<int64_t>(chunk, 1) > 1 || ngroups > 1;
    // tail split: a chunk's bulk kernels (unpack, classify, sort, first band level) on compute
    // stream k mod 2, its latency-bound rest (second level, wide level, exact kernel,
    // compaction) on one tail stream in chunk order, three scratch sets: chunk k + 2's bulk no
    // longer queues behind chunk k's tail (C5 pooled call 24.7 -> 21.6 ms, C2 unchanged).
    // (Chunk k's compaction waits for the copy of the runs a set back, ev_out[k - nsets],
    // recorded once the host has read that chunk's total: one set cannot pipeline chunks.)
    static_assert(kScratchSets >= 6 && kComputeStreams == 3, "the tail split needs three scratch sets (a dual call six)");
    const bool tail_split = several;
    // a dual call: three sets per pass (set k % 6 keeps a pass's chunks on its own sets), so a slow
    // pass-1 chunk never holds back the set a pass-0 chunk needs
    const int nsets = dual ? 6 : several ? 3 : 1;
    for (int si = 0; si < nsets && !rc; ++si) {
        c->s = &c->sc[si];
        configured = -1;
        for (int g = 0; g < ngroups && !rc; ++g) {
            const int64_t gn = groups ? (*groups->first)[(size_t)g + 1] - (*groups->first)[(size_t)g] : n;
            if (gn > 0 || ngroups == 1) rc = use_group(g, std::max<int64_t>(1, std::min(chunk, gn)));
            if (!rc && groups && si == nsets - 1 && gn > 0) {   // every set's buffers sized: keep the decisions
                gcfg[(size_t)g] = save_cfg(c);
                have_cfg[(size_t)g] = 1;
            }
        }
        if (!rc) rc = ops_reserve(c, chunk, dual ? 2 * n + 1 : n);
        // the fallback lists are indexed by the call's read (d_fallback + chunk base)
        if (!rc && (c->s->d_fallback.reserve((size_t)std::max<int64_t>(n, 1)) != hipSuccess ||
                    c->s->d_fallback2.reserve((size_t)std::max<int64_t>(n, 1)) != hipSuccess))
            rc = fail(c, NW_E_NOMEM, "device allocation failed for %lld reads", (long long)n);
    }
    ht.lap(1);
    if (ngroups > 1) configured = -1;   // the pipeline restores each group's saved configuration
    c->s = &c->sc[0];
    c->skip16 = false;
    const char* adapt = std::getenv("CRISPR_NW_ADAPT");   // "0": every chunk runs both band levels
    const bool adaptive = !(adapt && std::strcmp(adapt, "0") == 0);
    std::vector<char> one_level((size_t)std::max<int64_t>(nchunks, 1), 0);   // chunk ran the 32-diagonal level alone
    // (Rounds 3-5 ran a score-only diagonal pass over the reads of the amplicon's length ahead of
    // the first level's traceback fill in all but a call's last chunk, switched off per chunk when it
    // handed most reads on.  With round 6's classify certificates taking nearly all of those reads its
    // sweep only lengthened each chain: removed, in-process A/Bs C2 call 1.894 -> 1.833 ms, resident
    // pass 0.536 -> 0.484 ms, dual call 5.28 -> 5.12 ms, C1 shape 3.03 -> 2.98 ms)
    if (rc) {
        (void)hipStreamSynchronize(c->s_in);
        return restore(rc);
    }
    HIP_OR_FAIL(c, hipMemsetAsync(c->d_ctl64.p, 0, 2 * nw::kOpsCtlAll * sizeof(int64_t), c->stream));
    // copies of a known sequence from one alignment (packed classify): the caller's (nw_set_known),
    // or in a resident pass against a new amplicon the one the batch was last aligned against.  The
    // alignment runs on the upload stream of a resident pass (idle), else on the tail stream (its
    // first tail packet comes a chunk's chain later); every compaction waits for it
    c->known_on = false;
    c->kset[0].on = c->kset[1].on = false;
    if (dual) {   // each pass's copies of the other pass's amplicon
        for (int q = 0; q < 2 && n > 0; ++q) {
            if ((rc = use_group(q, std::min(chunk, n)))) return restore(rc);
            if (c->use_diag && (rc = known_prepare(c, (*groups->refs)[(size_t)(1 - q)], c->cstream[2], q)))
                return restore(rc);
        }
    } else {
        const std::string& K = (!c->known_seq.empty() && c->known_seq != c->ref) ? c->known_seq
                               : (!upload && c->resident_ref != c->ref) ? c->resident_ref : c->known_seq;
        const bool packed_classify = (pk != nullptr && upload) || (!upload && c->resident_packed);
        if (!groups && packed_classify && c->use_diag && n > 0 && !K.empty() && K != c->ref) {
            if ((rc = use_group(0, std::min(chunk, n))) || (rc = known_prepare(c, K, upload ? c->cstream[2] : c->s_in)))
                return restore(rc);
        }
    }
    // per pass: the caller's outputs, the runs' running total
    nw_stat* st_p[2] = {stats, dual ? dual->stats2 : nullptr};
    int64_t* oo_p[2] = {ops_off, dual ? dual->ops_off2 : nullptr};
    uint32_t* ops_p[2] = {ops_out, dual ? dual->ops_out2 : nullptr};
    const int64_t cap_p[2] = {ops_cap, dual ? dual->ops_cap2 : 0};
    int64_t total_p[2] = {0, 0};
    int64_t err = 0;
    bool cap_short = false;
    // Chunk k's runs go back once the host has read its total (copy_runs).  (Copying an
    // estimate of them as soon as the chunk is done measured no gain on the 1M-read call and a
    // loss on the pooled call's 96 small chunks: not kept.)
    // The last chunk's records, offsets and runs are written by its compaction kernel straight
    // into the caller's buffers when they are page-locked: no copies and no host round trip
    // after the call's last kernel (2.31 -> 2.27 ms per 1M-read call)
    const int last_pass = nchunks >= 1 ? chunks[(size_t)nchunks - 1].pass : 0;
    const bool direct_out = nchunks >= 1 && host_mapped(st_p[last_pass]) && host_mapped(oo_p[last_pass]) &&
                            (!ops_p[last_pass] || host_mapped(ops_p[last_pass]));
    // (The last two / three chunks writing their outputs the same way measured 1.968 vs 2.002 / 2.015 vs
    // 2.392 ms per C2 call in round 6: the PCIe writes then sit in those chunks' chains.  Not kept.)
    std::vector<char> direct_done((size_t)std::max<int64_t>(nchunks, 1), 0);
    auto copy_runs = [&](int64_t k) -> int {
        ht.lap(4);
        HIP_OR_FAIL(c, hipEventSynchronize(c->ev_ce[(size_t)k]));
        ht.lap(5);
        const int64_t* h = c->h_ctl + nw::kOpsCtl * k;
        err |= h[3];
        const int64_t cb = h[1], tot = h[2];
        const int pass = chunks[(size_t)k].pass;
        uint32_t* po = ops_p[pass];
        if (!po) {   // records only (a scores-only pass, CORE:1740-1741): the runs stay on the device
        } else if (cb + tot > cap_p[pass]) cap_short = true;
        else if (tot > 0 && !direct_done[(size_t)k])
            HIP_OR_FAIL(c, hipMemcpyAsync(po + cb, c->sc[k % nsets].d_staging.p, sizeof(uint32_t) * (size_t)tot,
                                          hipMemcpyDeviceToHost, c->s_out));
        HIP_OR_FAIL(c, hipEventRecord(c->ev_out[(size_t)k], c->s_out));
        total_p[pass] = cb + tot;
        if (po) c->ops_d2h_bytes += 4 * tot;
        return NW_OK;
    };
    c->ops_d2h_bytes = 0;
    int trace_chunks = 0;
    if (const char* e = std::getenv("CRISPR_NW_TRACE")) trace_chunks = std::atoi(e);
    c->trace_used = 0;
    // (a dual call: its pass's chunk two back -- the host never waits for the other pass's chunks)
    const int64_t lag = dual ? 4 : std::max(1, nsets - 1);
    // chunk k waits on ev_out[k - nsets], recorded by copy_runs(k - nsets) once k - nsets <= k' - lag for
    // an earlier k': every wait needs lag < nsets
    if (nchunks > nsets && lag >= nsets)
        return restore(fail(c, NW_E_INVALID, "ops call: run-copy lag must be below the scratch sets"));
    int64_t runs_queued = 0;   // chunks [0, runs_queued) had their runs copies queued early (the last iteration)
    bool any_diag = false;
    // a resident packed batch (nw_align_ops_resident after nw_align_ops_packed): the band path's
    // classify decodes it again; the exact kernels alone (-endweight, amplicons over 1024 bp)
    // need its bytes, unpacked once here before any chunk
    const bool packed_resident = !upload && c->resident_packed && c->use_diag;
    if (!upload && c->resident_packed && !c->use_diag && n > 0)
        HIP_OR_FAIL(c, nw::launch_unpack((const uint32_t*)c->d_packed.p, P0, base0, base0 + nbytes, c->d_exc_pos.p,
                                         c->d_exc_byte.p, 0, c->resident_n_exc, c->d_reads.p, c->reads_bias, c->stream));
    // the ctl reset and the exceptions' upload are on the first compute stream and s_in:
    // both compute streams start after them
    HIP_OR_FAIL(c, hipEventRecord(c->ev_start, c->stream));
    for (int k = 1; k < std::min(nsets, kComputeStreams); ++k)
        HIP_OR_FAIL(c, hipStreamWaitEvent(c->cstream[k], c->ev_start, 0));
    for (int64_t k = 0; k < nchunks; ++k) {
        const int64_t lo = chunks[(size_t)k].lo, hi = chunks[(size_t)k].hi;
        c->s = &c->sc[k % nsets];
        c->cs = c->cstream[k % std::min(nsets, kComputeStreams)];
        if (tail_split) {
            c->cs = c->cstream[k % 2];
            // the last chunks keep their tail on their own compute stream (no later chunk's bulk
            // queues behind it there): their tails overlap instead of queueing on the tail stream
            // (a one-amplicon call keeps each chunk's tail on its compute stream: in-process A/Bs,
            // C1 shape 5.05 -> 4.49 ms, C2 1.977 -> 1.958 ms; the pooled call's many small chunks and the
            // dual call keep the tail stream: 16.35 vs 19.14 ms, 5.34 vs 5.46 ms)
            c->split_to = groups ? c->cstream[2] : nullptr;
            c->split_ev = c->ev_bulk[(size_t)k];
            // the set's previous chunk (k - 3) must be through its tail
            if (k >= nsets) HIP_OR_FAIL(c, hipStreamWaitEvent(c->cs, c->ev_ce[(size_t)(k - nsets)], 0));
        }
        if (upload) HIP_OR_FAIL(c, hipStreamWaitEvent(c->cs, c->ev_in[(size_t)chunks[(size_t)k].up], 0));
        // (a timing event here sat in every chunk's chain: only with the host timing on)
        if (ht.on) HIP_OR_FAIL(c, hipEventRecord(c->ev_cs[(size_t)k], c->cs));
        if ((rc = use_group(chunks[(size_t)k].g, hi - lo))) return restore(rc);
        const int pass = chunks[(size_t)k].pass;
        c->out_off = pass ? n + 1 : 0;   // a dual call's pass 1: its records and run offsets after pass 0's
        c->ctl_pass = pass;
        c->kcur = dual ? pass : 0;
        c->known_on = c->kset[c->kcur].on;
        // the first level's lane walk + stop summary on chunks of >= 65536 reads of one
        // amplicon (in-process A/Bs, wave walk vs lane walk on every such chunk: C2 1.954 vs 1.961 ms,
        // C3 5.578 vs 5.570, C1 7.082 vs 7.070 -- the same -- while the kernel-resident pass of the
        // same kernels runs 0.81 -> 0.69 ms; the pooled call's 96 small chunks lost: 16.61 vs 17.15 ms)
        c->lane_call = (!groups || dual) && hi - lo >= 65536;
        c->pkc = nw::KernelArgs{};
        if (pk && upload && !c->use_diag) {   // the exact kernels read bytes: the chunk's bases -> bytes + exceptions
            const int64_t b0 = offsets[lo], b1 = offsets[hi];
            const int64_t e0 = std::lower_bound(pk->exc_pos, pk->exc_pos + pk->n_exc, b0) - pk->exc_pos;
            const int64_t e1 = std::lower_bound(pk->exc_pos, pk->exc_pos + pk->n_exc, b1) - pk->exc_pos;
            nw::LenSeg lsk{};
            if (lens_on)
                lsk = nw::LenSeg{(const uint16_t*)(c->d_lens.p + 8 * ngroups_len), (const int64_t*)c->d_lens.p,
                                 lo / nw::kLenGroup, hi / nw::kLenGroup - lo / nw::kLenGroup + 1, lo, hi, c->d_offsets.p};
            const nw::LenSeg* ls = lens_on ? &lsk : nullptr;
            HIP_OR_FAIL(c, nw::launch_unpack((const uint32_t*)c->d_packed.p, P0, b0, b1, c->d_exc_pos.p, c->d_exc_byte.p,
                                             e0, e1, c->d_reads.p, c->reads_bias, c->cs, ls));
        } else if ((pk && upload) || packed_resident) {
            // band path: classify decodes the chunk from the 2-bit stream itself (rebuilding its
            // offsets from the lengths) and writes only the bytes of the reads that need the DP --
            // no unpack launch, and 2 bits per base read instead of a byte written and re-read
            c->pkc.pk_words = (const uint32_t*)c->d_packed.p;
            c->pkc.pk_pos0 = 4 * P0;
            c->pkc.pk_exc_pos = c->d_exc_pos.p;
            c->pkc.pk_exc_byte = c->d_exc_byte.p;
            if (upload) {
                c->pkc.pk_e0 = std::lower_bound(pk->exc_pos, pk->exc_pos + pk->n_exc, offsets[lo]) - pk->exc_pos;
                c->pkc.pk_e1 = std::lower_bound(pk->exc_pos, pk->exc_pos + pk->n_exc, offsets[hi]) - pk->exc_pos;
            } else {
                c->pkc.pk_e0 = 0;
                c->pkc.pk_e1 = c->resident_n_exc;
            }
            if (lens_on) {
                c->pkc.pk_len = (const uint16_t*)(c->d_lens.p + 8 * ngroups_len);
                c->pkc.pk_gbase = (const int64_t*)c->d_lens.p;
            }
            c->pkc.pk_call_lo = lo;
        }
        any_diag = any_diag || c->use_diag;
        // adaptive first level: when most of the DP reads of the chunks done so far needed the
        // 32-diagonal level (e.g. the HDR pass: a 10-bp block substitution costs two 10-bp gaps
        // or 10 mismatches, beyond what 16 diagonals certify), the next chunks skip the
        // 16-diagonal level (its fill and walk would be spent on reads it hands on).  (The
        // converse -- sending the first level's give-ups straight to the exact kernel when few
        // reach the second level -- measured 3 % on C2 but is not safe to choose from earlier
        // chunks: with the HDR reads last (synth.c3_workload), the last chunks sent tens of
        // thousands of reads to the exact kernel, 15 -> 24 ms per C3 step.  The same choice
        // made on the device from the chunk's own count measured no gain: the skipped
        // level's launches remain.)
        // The newest chunk the host has read back (k - lag - 1, synchronised in copy_runs)
        // decides from its own counts when it ran both levels; while the level is skipped
        // every 4th chunk runs both again, so input that changes back is noticed.
        // (a dual call: its pass's own chunks; the passes' counts accumulate apart)
        static const int64_t zero[nw::kOpsCtl] = {};
        const int64_t jn = newest_same(k, lag + 1);
        const int64_t* hn = jn >= 0 ? c->h_ctl + nw::kOpsCtl * jn : zero;
        const int64_t* hpn = jn >= 0 && prev_same(jn) >= 0 ? c->h_ctl + nw::kOpsCtl * prev_same(jn) : zero;
        if (dual) c->skip16 = false;   // (each chunk decides for its own pass)
        if (adaptive && jn >= 0) {   // pooled calls too: one library's amplicons, one read source
            if (!one_level[(size_t)jn]) {
                const int64_t dp = (hn[6] - hn[7]) - (hpn[6] - hpn[7]), l2 = hn[5] - hpn[5];
                c->skip16 = dp >= 2048 && 2 * l2 > dp;
            } else {
                c->skip16 = (in_pass(k) & 3) != 0;
            }
        }
        one_level[(size_t)k] = c->skip16 && c->diag16_fill.grid > 0;
        // (No second-level launches while the newest chunk read back needed none -- the wide level
        // taking the whole redo list -- measured 1.926 vs 1.939 ms per C2 call but is not safe to
        // choose from earlier chunks: the C3 amplicon pass, whose HDR reads come last, sent ~30k of
        // them past the wide level's region to the exact kernel, 5.96 -> 14.5 ms per C3 step.  Lost
        // on C2 and not kept either: spinning on the chunk events, the last chunks' tails on their
        // own compute streams, explicit chunk ramps ending in small chunks, the last chunk's DP
        // reads straight to the wide level, the lane walk in the chunks (1.975 vs 1.959 ms; C3 14.50
        // vs 14.56), the 32-diagonal level's lane walk, the last chunk alone
        // on a high-priority stream, each chunk's upload split over two streams: +0.01 to +0.58 ms.)
        // the exact kernel's grid: small while the newest chunk read back sent it few reads
        // (after the wide level it gets the rare read no band certifies)
        c->exact_small = jn < 0 || hn[8] - hpn[8] < 256;
        // diagnostics: the last chunks' launches
        c->trace_on = trace_chunks > 0 && k >= nchunks - trace_chunks;
        c->trace_chunk = (int)k;
        // the compaction writes the chunk's ctl into h_ctl[k] itself
        nw::OpsHostOut ho{};
        const bool direct_k = direct_out && k == nchunks - 1;
        if (direct_k) ho = nw::OpsHostOut{(const int4*)(c->d_stats.p + c->out_off + lo), (int4*)(st_p[pass] + lo),
                                          oo_p[pass] + lo, ops_p[pass], ops_p[pass] ? cap_p[pass] : 0};
        // the compaction after its pass's previous one (the running base of the pass's ctl block)
        if ((rc = launch_range_ops(c, lo, k >= nsets ? c->ev_out[(size_t)(k - nsets)] : nullptr,
                                   prev_same(k) >= 0 ? c->ev_ce[(size_t)prev_same(k)] : nullptr,
                                   c->h_ctl + nw::kOpsCtl * k, (int)(in_pass(k) & 1), direct_k ? &ho : nullptr)))
            return restore(rc);
        direct_done[(size_t)k] = direct_k;
        HIP_OR_FAIL(c, hipEventRecord(c->ev_ce[(size_t)k], c->cs));
        // s_out order: chunk k - lag's runs (their size is known once that chunk is done:
        // the host waits for it, so lag = nsets - 1 chunks stay queued ahead), then chunk
        // k's records and offsets
        if (k >= lag && (rc = copy_runs(k - lag))) return restore(rc);
        // the last chunk: every earlier chunk's runs are queued ahead of its records, so they
        // copy while it computes (otherwise s_out would hold them behind the last chunk's end)
        if (k == nchunks - 1)
            for (int64_t j = std::max<int64_t>(0, k - lag + 1); j < k; ++j) {
                if ((rc = copy_runs(j))) return restore(rc);
                runs_queued = j + 1;
            }
        if (!direct_k) {
            HIP_OR_FAIL(c, hipStreamWaitEvent(c->s_out, c->ev_ce[(size_t)k], 0));
            HIP_OR_FAIL(c, hipMemcpyAsync(st_p[pass] + lo, c->d_stats.p + c->out_off + lo,
                                          sizeof(nw::Stat) * (size_t)(hi - lo), hipMemcpyDeviceToHost, c->s_out));
            HIP_OR_FAIL(c, hipMemcpyAsync(oo_p[pass] + lo, c->d_opsoff.p + c->out_off + lo,
                                          sizeof(int64_t) * (size_t)(hi - lo), hipMemcpyDeviceToHost, c->s_out));
        }
        c->ops_d2h_bytes += (int64_t)(sizeof(nw::Stat) + sizeof(int64_t)) * (hi - lo);
    }
    for (int64_t k = std::max<int64_t>(runs_queued, nchunks - lag); k < nchunks; ++k)
        if ((rc = copy_runs(k))) return restore(rc);
    ht.lap(4);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->s_out));
    ht.lap(6);
    ops_off[n] = total_p[0];
    if (dual) dual->ops_off2[n] = total_p[1];
    if (nchunks > 0) {   // the call's reads by path (nw_batch_path_counts / nw_batch_fallbacks; a dual call: pass 0's)
        int64_t kl = nchunks - 1;   // the last chunk of pass 0 (a dual call interleaves the passes)
        while (kl > 0 && chunks[(size_t)kl].pass != 0) --kl;
        const int64_t* h = c->h_ctl + nw::kOpsCtl * kl;
        const bool two = any_diag && c->diag16_fill.grid > 0;
        c->call_counts[0] = any_diag ? n - h[6] : 0;
        c->call_counts[1] = two ? h[6] - h[7] : 0;                // first level: two-level chunks' DP reads
        c->call_counts[2] = any_diag ? (two ? h[5] + h[7] : h[6]) : 0;
        c->call_counts[3] = h[4];
        c->call_exact = h[8];
    }
    c->call_done = true;
    // device times: the upload span on s_in, the chunks' compute spans summed
    c->ops_h2d_ms = 0.0f;
    c->ops_compute_ms = 0.0f;
    c->ops_h2d_bytes = upload ? h2d_bytes : 0;
    if (nchunks > 0) {
        if (upload)
            HIP_OR_FAIL(c, hipEventElapsedTime(&c->ops_h2d_ms, c->ev_h0, c->ev_h1));
        // the chunks' compute spans summed (host timing on: their start events), else the call's device
        // span, first upload to the last chunk's end
        for (int64_t k = 0; k < nchunks; ++k) {
            float ms = 0.0f;
            if (ht.on) HIP_OR_FAIL(c, hipEventElapsedTime(&ms, c->ev_cs[(size_t)k], c->ev_ce[(size_t)k]));
            c->ops_compute_ms += ms;
        }
        if (!ht.on) HIP_OR_FAIL(c, hipEventElapsedTime(&c->ops_compute_ms, c->ev_h0, c->ev_ce[(size_t)nchunks - 1]));
        for (size_t i = 0; i < c->trace_used; ++i) {
            float t = 0;
            (void)hipEventElapsedTime(&t, c->ev_h0, c->trace_ev[i].second);
            std::fprintf(stderr, "  trace chunk %s: %.1f us\n", c->trace_ev[i].first.c_str(), 1e3 * t);
        }
        c->trace_on = false;
        c->trace_used = 0;
        if (ht.on)   // per chunk (ms from the first upload): upload done, compute start, compute end
            for (int64_t k = 0; k < nchunks; ++k) {
                float a = 0, b = 0, e = 0;
                (void)a;   // (the uploads' events do not time: ev_h1 is the last one's end)
                (void)hipEventElapsedTime(&b, c->ev_h0, c->ev_cs[(size_t)k]);
                (void)hipEventElapsedTime(&e, c->ev_h0, c->ev_ce[(size_t)k]);
                std::fprintf(stderr, "  chunk %lld [%lld reads]: in %.3f start %.3f end %.3f\n", (long long)k,
                             (long long)(chunks[(size_t)k].hi - chunks[(size_t)k].lo), a, b, e);
            }
    }
    c->resident_ok = true;   // the batch stays in HBM for nw_align_ops_resident
    if (upload) {
        c->resident_packed = pk != nullptr;
        c->resident_n_exc = pk ? pk->n_exc : 0;
    }
    c->resident_n = n;
    c->resident_lo = base0;
    c->resident_hi = base0 + nbytes;
    c->resident_ref = groups ? std::string() : c->ref;   // a later resident pass's known sequence
    if ((rc = ops_error(c, err))) return restore(rc);
    if (cap_short)
        return restore(fail(c, NW_E_CAPACITY, "ops_cap %lld < %lld runs (ops_off holds the offsets)",
                            (long long)(total_p[0] > ops_cap ? ops_cap : cap_p[1]),
                            (long long)(total_p[0] > ops_cap ? total_p[0] : total_p[1])));
    return restore(NW_OK);
}

}  // namespace

extern "C" {

int nw_align_ops(nw_ctx* c, const char* reads, const int64_t* offsets, int64_t n, uint32_t* ops_out, int64_t ops_cap,
                 int64_t* ops_off, nw_stat* stats) {
    return ops_call(c, reads, offsets, n, ops_out, ops_cap, ops_off, stats, true);
}

int nw_align_ops_packed(nw_ctx* c, const uint8_t* packed, const int64_t* offsets, int64_t n, const int64_t* exc_pos,
                        const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out, int64_t ops_cap, int64_t* ops_off,
                        nw_stat* stats) {
    if (n_exc < 0) return fail(c, NW_E_INVALID, "bad exception count");
    const PackedInput pk{packed, exc_pos, exc_byte, n_exc};
    return ops_call(c, nullptr, offsets, n, ops_out, ops_cap, ops_off, stats, true, nullptr, &pk);
}

int nw_align_ops_packed_lens(nw_ctx* c, const uint8_t* packed, const int64_t* offsets, const uint16_t* lens, int64_t n,
                             const int64_t* exc_pos, const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out,
                             int64_t ops_cap, int64_t* ops_off, nw_stat* stats) {
    if (n_exc < 0) return fail(c, NW_E_INVALID, "bad exception count");
    if (n > 0 && !lens) return fail(c, NW_E_INVALID, "no lengths");
    PackedInput pk{packed, exc_pos, exc_byte, n_exc};
    pk.lens = lens;
    return ops_call(c, nullptr, offsets, n, ops_out, ops_cap, ops_off, stats, true, nullptr, &pk);
}

int nw_align_ops_resident(nw_ctx* c, const int64_t* offsets, int64_t n, uint32_t* ops_out, int64_t ops_cap,
                          int64_t* ops_off, nw_stat* stats) {
    return ops_call(c, nullptr, offsets, n, ops_out, ops_cap, ops_off, stats, false);
}

// Pooled batch, ops output (CRISPRessoPooled.py:882-908 runs one CRISPResso -- one
// needle per pass -- per amplicon): one call, every amplicon's tables uploaded once,
// chunks of one amplicon each pipelined as in nw_align_ops.  Reads grouped by
// amplicon (ref_of_read non-decreasing, as the demultiplexed per-amplicon read sets
// arrive) are used in place; otherwise they are grouped on the host first and the
// outputs put back in the caller's order.
}  // extern "C"

namespace {

int multi_ops(nw_ctx* c, const char* refs, const int64_t* ref_offsets, int32_t n_refs, const char* reads,
              const int64_t* offsets, const int32_t* ref_of_read, int64_t n, uint32_t* ops_out, int64_t ops_cap,
              int64_t* ops_off, nw_stat* stats, const PackedInput* pk) {
    if (!c) return NW_E_INVALID;
    HostTimer ht("index-scan tables");
    if (n_refs <= 0 || !refs || !ref_offsets) return fail(c, NW_E_INVALID, "no amplicons");
    if (n < 0 || (n > 0 && (!(reads || pk) || !offsets || !ref_of_read || !stats)) || !ops_off)
        return fail(c, NW_E_INVALID, "bad batch");
    std::vector<std::string> amps((size_t)n_refs);
    for (int32_t g = 0; g < n_refs; ++g) {
        const int64_t L = ref_offsets[g + 1] - ref_offsets[g];
        if (L <= 0 || L > kMaxRef) return fail(c, NW_E_UNSUPPORTED, "amplicon %d has length %lld", g, (long long)L);
        amps[(size_t)g].assign(refs + ref_offsets[g], refs + ref_offsets[g + 1]);
    }
    (void)hipSetDevice(c->device);
    // reads per amplicon and whether the reads come grouped: per part of the host pool
    // (memory-bound), a bad index located afterwards
    std::vector<int64_t> first((size_t)n_refs + 1, 0);
    bool grouped = true;
    {
        nw_host::Pool& pool = nw_host::Pool::get();
        const int parts = (int)std::min<int64_t>(pool.threads(), std::max<int64_t>(1, n >> 17));
        std::vector<std::vector<int64_t>> cnt((size_t)parts);
        std::vector<char> pbad((size_t)parts, 0), psorted((size_t)parts, 1);
        pool.run(parts, [&](int q) {
            int64_t lo, hi;
            nw_host::Pool::range(n, parts, q, &lo, &hi);
            std::vector<int64_t>& h = cnt[(size_t)q];
            h.assign((size_t)n_refs + 1, 0);
            uint32_t bad = 0, desc = 0;
            for (int64_t r = lo; r < hi; ++r) {
                const int32_t g = ref_of_read[r];
                const bool out = (uint32_t)g >= (uint32_t)n_refs;
                bad |= out;
                ++h[out ? (size_t)n_refs : (size_t)g];
                desc |= r > lo && g < ref_of_read[r - 1];
            }
            pbad[(size_t)q] = bad != 0;
            psorted[(size_t)q] = desc == 0 && (lo == 0 || hi == lo || ref_of_read[lo] >= ref_of_read[lo - 1]);
        });
        for (int q = 0; q < parts; ++q)
            if (pbad[(size_t)q])
                for (int64_t r = 0; r < n; ++r)
                    if ((uint32_t)ref_of_read[r] >= (uint32_t)n_refs)
                        return fail(c, NW_E_INVALID, "read %lld has amplicon index %d", (long long)r, ref_of_read[r]);
        for (int q = 0; q < parts; ++q) {
            grouped = grouped && psorted[(size_t)q];
            for (int32_t g = 0; g < n_refs; ++g) first[(size_t)g + 1] += cnt[(size_t)q][(size_t)g];
        }
    }
    for (int32_t g = 0; g < n_refs; ++g) first[(size_t)g + 1] += first[(size_t)g];
    ht.lap(0);
    int rc = upload_shared(c);
    std::vector<Profile> profs;
    if (!rc) rc = upload_profiles(c, amps, &profs);
    if (rc) return rc;
    ht.lap(1);
    c->ref.clear();   // the context has no single amplicon afterwards (nw_set_reference again)
    c->cur = Profile{};
    Groups grp{&amps, &profs, &first};
    if (grouped) {
        rc = ops_call(c, reads, offsets, n, ops_out, ops_cap, ops_off, stats, true, &grp, pk);
        c->ref.clear();
        c->cur = Profile{};
        return rc;
    }
    if (pk) return fail(c, NW_E_INVALID, "packed pooled batches must be grouped by amplicon (ref_of_read ascending)");
    // group on the host (stable), align, then back to the caller's order
    std::vector<int64_t> order((size_t)n), fill(first.begin(), first.end() - 1);
    for (int64_t r = 0; r < n; ++r) order[(size_t)fill[(size_t)ref_of_read[r]]++] = r;
    std::vector<int64_t> soff((size_t)n + 1, 0);
    for (int64_t s2 = 0; s2 < n; ++s2)
        soff[(size_t)s2 + 1] = soff[(size_t)s2] + (offsets[order[(size_t)s2] + 1] - offsets[order[(size_t)s2]]);
    std::vector<char> sreads((size_t)std::max<int64_t>(soff[(size_t)n], 1));
    for (int64_t s2 = 0; s2 < n; ++s2) {
        const int64_t r = order[(size_t)s2];
        std::memcpy(sreads.data() + soff[(size_t)s2], reads + offsets[r], (size_t)(offsets[r + 1] - offsets[r]));
    }
    std::vector<nw::Stat> sst((size_t)std::max<int64_t>(n, 1));
    std::vector<int64_t> sopo((size_t)n + 1);
    std::vector<uint32_t> sops((size_t)std::max<int64_t>(ops_out ? std::max<int64_t>(ops_cap, 0) : 0, 1));
    rc = ops_call(c, sreads.data(), soff.data(), n, ops_out ? sops.data() : nullptr, ops_out ? ops_cap : 0,
                  sopo.data(), (nw_stat*)sst.data(), true, &grp);
    c->ref.clear();
    c->cur = Profile{};
    if (rc && rc != NW_E_CAPACITY) return rc;
    // caller order: records, run counts -> offsets, runs
    std::vector<int64_t> cnt((size_t)n);
    for (int64_t s2 = 0; s2 < n; ++s2) {
        const int64_t r = order[(size_t)s2];
        std::memcpy(&stats[r], &sst[(size_t)s2], sizeof(nw::Stat));
        cnt[(size_t)r] = sopo[(size_t)s2 + 1] - sopo[(size_t)s2];
    }
    ops_off[0] = 0;
    for (int64_t r = 0; r < n; ++r) ops_off[r + 1] = ops_off[r] + cnt[(size_t)r];
    if (rc == NW_E_CAPACITY) return rc;
    if (ops_out)
        for (int64_t s2 = 0; s2 < n; ++s2) {
            const int64_t r = order[(size_t)s2];
            std::memcpy(ops_out + ops_off[r], sops.data() + sopo[(size_t)s2], sizeof(uint32_t) * (size_t)cnt[(size_t)r]);
        }
    return NW_OK;
}

}  // namespace

extern "C" {

int nw_align_multi_ops(nw_ctx* c, const char* refs, const int64_t* ref_offsets, int32_t n_refs, const char* reads,
                       const int64_t* offsets, const int32_t* ref_of_read, int64_t n, uint32_t* ops_out, int64_t ops_cap,
                       int64_t* ops_off, nw_stat* stats) {
    return multi_ops(c, refs, ref_offsets, n_refs, reads, offsets, ref_of_read, n, ops_out, ops_cap, ops_off, stats,
                     nullptr);
}

int nw_align_multi_ops_packed(nw_ctx* c, const char* refs, const int64_t* ref_offsets, int32_t n_refs,
                              const uint8_t* packed, const int64_t* offsets, const int32_t* ref_of_read, int64_t n,
                              const int64_t* exc_pos, const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out,
                              int64_t ops_cap, int64_t* ops_off, nw_stat* stats) {
    if (!c) return NW_E_INVALID;
    if (n_exc < 0 || (n > 0 && !packed)) return fail(c, NW_E_INVALID, "bad packed batch");
    const PackedInput pk{packed, exc_pos, exc_byte, n_exc};
    return multi_ops(c, refs, ref_offsets, n_refs, nullptr, offsets, ref_of_read, n, ops_out, ops_cap, ops_off, stats,
                     &pk);
}

int nw_align_multi_ops_packed_lens(nw_ctx* c, const char* refs, const int64_t* ref_offsets, int32_t n_refs,
                                   const uint8_t* packed, const int64_t* offsets, const uint16_t* lens,
                                   const int32_t* ref_of_read, int64_t n, const int64_t* exc_pos, const uint8_t* exc_byte,
                                   int64_t n_exc, uint32_t* ops_out, int64_t ops_cap, int64_t* ops_off, nw_stat* stats) {
    if (!c) return NW_E_INVALID;
    if (n_exc < 0 || (n > 0 && (!packed || !lens))) return fail(c, NW_E_INVALID, "bad packed batch");
    PackedInput pk{packed, exc_pos, exc_byte, n_exc};
    pk.lens = lens;
    return multi_ops(c, refs, ref_offsets, n_refs, nullptr, offsets, ref_of_read, n, ops_out, ops_cap, ops_off, stats,
                     &pk);
}

int nw_align_dual_ops_packed_lens(nw_ctx* c, const char* ref2, int32_t ref2_len, const uint8_t* packed,
                                  const int64_t* offsets, const uint16_t* lens, int64_t n, const int64_t* exc_pos,
                                  const uint8_t* exc_byte, int64_t n_exc, uint32_t* ops_out, int64_t ops_cap,
                                  int64_t* ops_off, nw_stat* stats, uint32_t* ops_out2, int64_t ops_cap2,
                                  int64_t* ops_off2, nw_stat* stats2) {
    if (!c) return NW_E_INVALID;
    if (c->ref.empty()) return fail(c, NW_E_STATE, "nw_set_reference must come first");
    if (!ref2 || ref2_len <= 0) return fail(c, NW_E_INVALID, "empty second amplicon");
    if (ref2_len > kMaxRef) return fail(c, NW_E_UNSUPPORTED, "amplicon length %d exceeds %d", ref2_len, kMaxRef);
    if (n_exc < 0 || (n > 0 && (!packed || !lens || !stats2 || !ops_off2))) return fail(c, NW_E_INVALID, "bad packed batch");
    (void)hipSetDevice(c->device);
    PackedInput pk{packed, exc_pos, exc_byte, n_exc};
    pk.lens = lens;
    const std::string ref0 = c->ref;
    std::vector<std::string> amps{ref0, std::string(ref2, ref2 + ref2_len)};
    std::vector<Profile> profs;
    int rc = upload_shared(c);
    if (!rc) rc = upload_profiles(c, amps, &profs);
    if (rc) return rc;
    const std::vector<int64_t> first{0, n, 2 * n};
    Groups grp{&amps, &profs, &first};
    const Dual d{ops_out2, ops_cap2, ops_off2, stats2};
    rc = ops_call(c, nullptr, offsets, n, ops_out, ops_cap, ops_off, stats, true, &grp, &pk, &d);
    c->ref = ref0;   // the context keeps its amplicon (the arena holds both tables)
    c->cur = profs[0];
    return rc;
}

int nw_ops_times(const nw_ctx* c, float* h2d_ms, float* compute_ms, int64_t* h2d_bytes, int64_t* d2h_bytes) {
    if (!c) return NW_E_INVALID;
    if (h2d_ms) *h2d_ms = c->ops_h2d_ms;
    if (compute_ms) *compute_ms = c->ops_compute_ms;
    if (h2d_bytes) *h2d_bytes = c->ops_h2d_bytes;
    if (d2h_bytes) *d2h_bytes = c->ops_d2h_bytes;
    return NW_OK;
}

int nw_host_threads(void) { return nw_host::Pool::get().threads(); }

int nw_set_known(nw_ctx* c, const char* seq, int32_t len) {
    if (!c || len < 0 || (len > 0 && !seq)) return NW_E_INVALID;
    c->known_seq.assign(seq ? seq : "", (size_t)len);
    return NW_OK;
}

int nw_batch_set_phase_events(nw_ctx* c, int on) {
    if (!c) return NW_E_INVALID;
    c->phase_events = on != 0;
    return NW_OK;
}

int nw_batch_set_lane_walk(nw_ctx* c, int on) {
    if (!c) return NW_E_INVALID;
    c->lane_walk = on != 0;
    return NW_OK;
}

int nw_host_alloc(int64_t bytes, void** out) {
    if (!out || bytes < 0) return NW_E_INVALID;
    *out = nullptr;
    return hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault) == hipSuccess ? NW_OK
                                                                                                     : NW_E_NOMEM;
}

void nw_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int nw_host_register(void* p, int64_t bytes) {
    if (!p || bytes <= 0) return NW_E_INVALID;
    return hipHostRegister(p, (size_t)bytes, hipHostRegisterDefault) == hipSuccess ? NW_OK : NW_E_HIP;
}

int nw_host_unregister(void* p) {
    if (!p) return NW_E_INVALID;
    return hipHostUnregister(p) == hipSuccess ? NW_OK : NW_E_HIP;
}

int nw_batch_phase_times(nw_ctx* c, float* ms5) {
    if (!c || !ms5) return NW_E_INVALID;
    if (!c->ran) return fail(c, NW_E_STATE, "nothing has run");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 5; ++k) ms5[k] = 0.0f;
    if (!c->phases_recorded) return fail(c, NW_E_STATE, "the last run recorded no phase events (nw_batch_set_phase_events)");
    if (!c->use_diag || c->n <= 0) {
        HIP_OR_FAIL(c, hipEventElapsedTime(&ms5[4], c->ev0, c->ev1));
        return NW_OK;
    }
    const bool two = c->diag16_fill.grid > 0;
    HIP_OR_FAIL(c, hipEventElapsedTime(&ms5[0], c->ev0, c->ev_sort));
    HIP_OR_FAIL(c, hipEventElapsedTime(&ms5[1], c->ev_sort, c->ev_fill));
    HIP_OR_FAIL(c, hipEventElapsedTime(&ms5[2], c->ev_fill, c->ev_walk));
    HIP_OR_FAIL(c, hipEventElapsedTime(&ms5[3], c->ev_walk, c->ev_l2));
    HIP_OR_FAIL(c, hipEventElapsedTime(&ms5[4], c->ev_l2, c->ev1));
    if (!two) {   // one level: ms5[1..2] are the 32-diagonal level's, ms5[3] is empty
        ms5[3] = 0.0f;
    }
    return NW_OK;
}

int nw_batch_path_counts(nw_ctx* c, int64_t* counts4) {
    if (!c || !counts4) return NW_E_INVALID;
    if (c->call_done) {
        for (int k = 0; k < 4; ++k) counts4[k] = c->call_counts[k];
        return NW_OK;
    }
    if (!c->ran) return fail(c, NW_E_STATE, "nothing has run");
    (void)hipSetDevice(c->device);
    HIP_OR_FAIL(c, hipStreamSynchronize(c->stream));
    for (int k = 0; k < 4; ++k) counts4[k] = 0;
    if (!c->use_diag) {
        counts4[3] = nw_batch_fallbacks(c);
        return NW_OK;
    }
    int32_t fb[8] = {0, 0, 0, 0, 0, 0, 0, 0}, need = 0;
    HIP_OR_FAIL(c, hipMemcpy(fb, c->s->d_fallback_count.p, sizeof fb, hipMemcpyDeviceToHost));
    need = fb[1];   // the sort's DP count
    const bool two = c->diag16_fill.grid > 0;
    counts4[0] = c->n - need;             // exact copies (no DP)
    counts4[1] = two ? need : 0;          // first level (16 diagonals)
    // a skipped second level (KernelArgs::redo_direct) sent its reads to the exact kernel
    const bool direct = two && c->redo_direct > 0 && fb[2] <= c->redo_direct;
    counts4[2] = two ? (direct ? 0 : fb[2]) : need;   // second level (32 diagonals)
    counts4[3] = fb[0] + (direct ? fb[2] : 0);        // the 16 / 32 levels' give-ups (wide level + exact kernel)
    return NW_OK;
}

int64_t nw_batch_exact_reads(nw_ctx* c) {
    if (c && c->call_done) return c->call_exact;
    if (!c || !c->ran) return -1;
    if (!c->use_diag || c->wide_fill.grid <= 0) return nw_batch_fallbacks(c);
    (void)hipSetDevice(c->device);
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    int32_t fb[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpy(fb, c->s->d_fallback_count.p, sizeof fb, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    return fb[6];
}

}  // extern "C"
