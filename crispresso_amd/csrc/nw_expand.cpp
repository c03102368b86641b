// nw_expand.cpp -- host expansion of the ops output into alignment rows.
//
// nw_align_ops returns every read's traceback as runs (include/crispr_nw.h); the
// rows EMBOSS needle prints -- aligned amplicon, markup, aligned read, the strings
// parse_needle_output slices out of the srspair block (CRISPRessoCORE.py:1747-1754)
// -- are a function of the runs and the two sequences.  This builds them exactly as
// the kernels do in NW_OUT_ROWS mode (nw_common.h emit_alignment):
//   M column: '|' when the residues are equal ignoring case, ':' when EDNAFULL scores
//             the pair > 0, '.' otherwise; a '-' already in the input (RC-retry reads,
//             CORE:1846) is printed as is with markup ' ';
//   X / Y column: '-' opposite the residue, markup ' '.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/crispr_nw.h"
#include "host_pool.h"
#include "nw_edna.h"

namespace {

struct Tables {
    unsigned char up[256];
    uint8_t code[256];
    bool pos[17][256];   // EDNAFULL(code a, byte b) > 0
    Tables() {
        for (int b = 0; b < 256; ++b) {
            up[b] = (unsigned char)std::toupper(b);
            code[b] = nw::code_of((unsigned char)b);
        }
        for (int a = 0; a < 17; ++a)
            for (int b = 0; b < 256; ++b) pos[a][b] = a < 16 && code[b] < 16 && nw::kEdna[a][code[b]] > 0;
    }
};

const Tables& tables() {
    static const Tables t;
    return t;
}

// one read; false when the runs do not cover both sequences or overflow the row
bool expand_one(const Tables& T, const unsigned char* ref, int64_t La, const uint8_t* acode, const unsigned char* rd,
                int64_t Lb, const uint32_t* ops, int64_t nops, char* o0, int64_t stride) {
    char* o1 = o0 + stride;
    char* o2 = o1 + stride;
    int64_t col = 0, ia = 0, jb = 0;
    for (int64_t q = 0; q < nops; ++q) {
        const uint32_t type = NW_RUN_TYPE(ops[q]);
        const int64_t len = NW_RUN_LEN(ops[q]);
        if (col + len > stride) return false;
        if (type == NW_RUN_M) {
            if (ia + len > La || jb + len > Lb) return false;
            std::memcpy(o0 + col, ref + ia, (size_t)len);
            std::memcpy(o2 + col, rd + jb, (size_t)len);
            for (int64_t k = 0; k < len; ++k) {
                const unsigned char ca = ref[ia + k], cb = rd[jb + k];
                char mk = '|';
                if (ca != cb || ca == '-') {
                    if (ca == '-' || cb == '-') mk = ' ';
                    else if (T.up[ca] == T.up[cb]) mk = '|';
                    else mk = T.pos[acode[ia + k]][cb] ? ':' : '.';
                }
                o1[col + k] = mk;
            }
            ia += len;
            jb += len;
        } else if (type == NW_RUN_X) {
            if (jb + len > Lb) return false;
            std::memset(o0 + col, '-', (size_t)len);
            std::memset(o1 + col, ' ', (size_t)len);
            std::memcpy(o2 + col, rd + jb, (size_t)len);
            jb += len;
        } else if (type == NW_RUN_Y) {
            if (ia + len > La) return false;
            std::memcpy(o0 + col, ref + ia, (size_t)len);
            std::memset(o1 + col, ' ', (size_t)len);
            std::memset(o2 + col, '-', (size_t)len);
            ia += len;
        } else {
            return false;
        }
        col += len;
    }
    return ia == La && jb == Lb;
}

}  // namespace

template <class F>
void parallel_for(int64_t n, int32_t nthreads, const F& f) {
    int nt = nthreads > 0 ? nthreads : nw_host::default_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n / 4096 + 1));
    if (nt == 1) {
        f(0, n);
        return;
    }
    std::vector<std::thread> pool;
    const int64_t per = (n + nt - 1) / nt;
    for (int t = 0; t < nt; ++t) {
        const int64_t lo = t * per, hi = std::min(n, lo + per);
        if (lo < hi) pool.emplace_back(f, lo, hi);
    }
    for (auto& th : pool) th.join();
}

extern "C" int nw_expand_ops_subset(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets,
                                    const int64_t* idx, int64_t m, const uint32_t* ops, const int64_t* ops_off,
                                    char* aln_out, int64_t stride, int32_t nthreads) {
    if (m < 0 || ref_len <= 0 || !ref || (m > 0 && (!reads || !offsets || !idx || !ops_off || !aln_out)))
        return NW_E_INVALID;
    const Tables& T = tables();
    std::vector<uint8_t> acode((size_t)ref_len);
    for (int32_t i = 0; i < ref_len; ++i) acode[(size_t)i] = T.code[(unsigned char)ref[i]];
    std::atomic<int> bad{0};
    parallel_for(m, nthreads, [&](int64_t lo, int64_t hi) {
        for (int64_t q = lo; q < hi; ++q) {
            const int64_t r = idx[q];
            const int64_t Lb = offsets[r + 1] - offsets[r];
            const int64_t k0 = ops_off[r], k1 = ops_off[r + 1];
            if (Lb == 0 && k1 == k0) continue;
            if (k1 < k0 || !ops ||
                !expand_one(T, (const unsigned char*)ref, ref_len, acode.data(), (const unsigned char*)reads + offsets[r],
                            Lb, ops + k0, k1 - k0, aln_out + q * 3 * stride, stride))
                bad.store(1, std::memory_order_relaxed);
        }
    });
    return bad.load() ? NW_E_INVALID : NW_OK;
}

// The rows of reads idx[0..m) concatenated column by column (read q's row in
// [row_off[q], row_off[q + 1]) of each buffer: its first row_off[q + 1] - row_off[q]
// columns, the `awidth` cut of parse_needle_output's first line), the non-'-' bytes of
// its read row in that span (the "length" column, CORE:1750) and whether its amplicon
// row is the amplicon itself (no read-side gap column: every such row can share one
// string).  What ops_to_dataframe builds its string columns from in one pass.  A read
// byte outside ASCII is an error (the columns are str; the FASTQ reader keeps letters).
extern "C" int nw_ops_rows_concat(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets,
                                  const int64_t* idx, int64_t m, const uint32_t* ops, const int64_t* ops_off,
                                  const int64_t* row_off, char* ref_rows, char* markup_rows, char* read_rows,
                                  int32_t* read_chars, uint8_t* ref_is_amplicon, int32_t nthreads) {
    if (m < 0 || ref_len <= 0 || !ref ||
        (m > 0 && (!reads || !offsets || !idx || !ops_off || !row_off || !ref_rows || !markup_rows || !read_rows ||
                   !read_chars || !ref_is_amplicon)))
        return NW_E_INVALID;
    const Tables& T = tables();
    std::vector<uint8_t> acode((size_t)ref_len);
    for (int32_t i = 0; i < ref_len; ++i) acode[(size_t)i] = T.code[(unsigned char)ref[i]];
    std::atomic<int> bad{0};
    parallel_for(m, nthreads, [&](int64_t lo, int64_t hi) {
        std::vector<char> tmp;
        for (int64_t q = lo; q < hi; ++q) {
            const int64_t r = idx[q];
            const int64_t Lb = offsets[r + 1] - offsets[r];
            const int64_t k0 = ops_off[r], k1 = ops_off[r + 1];
            const int64_t cols = row_off[q + 1] - row_off[q];
            int64_t aln = 0;
            bool gap_in_ref = false;
            for (int64_t k = k0; k < k1; ++k) {
                aln += NW_RUN_LEN(ops[k]);
                gap_in_ref |= NW_RUN_TYPE(ops[k]) == NW_RUN_X;
            }
            if (k1 < k0 || cols < 0 || cols > aln || (k1 > k0 && !ops)) {
                bad.store(1, std::memory_order_relaxed);
                continue;
            }
            if ((int64_t)tmp.size() < 3 * aln) tmp.resize((size_t)(3 * aln));
            if (aln > 0 && !expand_one(T, (const unsigned char*)ref, ref_len, acode.data(),
                                       (const unsigned char*)reads + offsets[r], Lb, ops + k0, k1 - k0, tmp.data(),
                                       aln)) {
                bad.store(1, std::memory_order_relaxed);
                continue;
            }
            const int64_t o = row_off[q];
            std::memcpy(ref_rows + o, tmp.data(), (size_t)cols);
            std::memcpy(markup_rows + o, tmp.data() + aln, (size_t)cols);
            const char* rr = tmp.data() + 2 * aln;
            std::memcpy(read_rows + o, rr, (size_t)cols);
            int32_t nc = 0;
            unsigned char hi = 0;
            for (int64_t k = 0; k < cols; ++k) {
                nc += rr[k] != '-';
                hi |= (unsigned char)rr[k];
            }
            if (hi & 0x80) bad.store(1, std::memory_order_relaxed);   // the columns are ASCII strings
            read_chars[q] = nc;
            ref_is_amplicon[q] = (uint8_t)(!gap_in_ref && cols == aln && aln == ref_len);
        }
    });
    return bad.load() ? NW_E_INVALID : NW_OK;
}

extern "C" int64_t nw_reads_equal_ref(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets,
                                      int64_t n, uint8_t* equal, int32_t nthreads) {
    if (n < 0 || !ref || (n > 0 && (!reads || !offsets || !equal))) return NW_E_INVALID;
    std::atomic<int64_t> count{0};
    parallel_for(n, nthreads, [&](int64_t lo, int64_t hi) {
        int64_t c = 0;
        for (int64_t r = lo; r < hi; ++r) {
            const bool e = offsets[r + 1] - offsets[r] == ref_len &&
                           std::memcmp(reads + offsets[r], ref, (size_t)ref_len) == 0;
            equal[r] = (uint8_t)e;
            c += e;
        }
        count += c;
    });
    return count.load();
}

namespace {

uint64_t read_hash(const unsigned char* p, int64_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    int64_t k = 0;
    for (; k + 8 <= n; k += 8) {
        uint64_t w;
        std::memcpy(&w, p + k, 8);
        h = (h ^ w) * 0xFF51AFD7ED558CCDull;
        h ^= h >> 32;
    }
    uint64_t w = 0;
    std::memcpy(&w, p + k, (size_t)(n - k));
    h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
    return h ^ (h >> 29);
}

}  // namespace

// rep[q] = the first q' with read idx[q']'s bytes equal to read idx[q]'s (idx null: the reads
// 0 .. m).  Hashes in parallel, then one open-addressing
// table per hash partition (each thread owns the reads whose hash falls in its partition,
// visited in read order, so the first occurrence is the one kept); equal hashes are
// confirmed by comparing the bytes.  Returns the number of distinct reads.
extern "C" int64_t nw_reads_first_copy(const char* reads, const int64_t* offsets, const int64_t* idx, int64_t n,
                                       int64_t* rep, int32_t nthreads) {
    if (n < 0 || (n > 0 && (!reads || !offsets || !rep))) return NW_E_INVALID;
    auto rd = [&](int64_t q) { return idx ? idx[q] : q; };
    if (n == 0) return 0;
    nw_host::Pool& pool = nw_host::Pool::get();
    int P = nthreads > 0 ? std::min(nthreads, pool.threads()) : pool.threads();
    P = (int)std::max<int64_t>(1, std::min<int64_t>(P, n / 8192 + 1));
    std::vector<uint64_t> h((size_t)n);
    pool.run(P, [&](int k) {
        int64_t lo, hi;
        nw_host::Pool::range(n, P, k, &lo, &hi);
        for (int64_t q = lo; q < hi; ++q) {
            const int64_t r = rd(q);
            h[(size_t)q] = read_hash((const unsigned char*)reads + offsets[r], offsets[r + 1] - offsets[r]);
        }
    });
    std::vector<int64_t> distinct((size_t)P, 0);
    pool.run(P, [&](int part) {
        // this partition's reads: hash % P == part (the slot comes from the high bits)
        int64_t cnt = 0;
        for (int64_t r = 0; r < n; ++r) cnt += (int)(h[(size_t)r] % (uint64_t)P) == part;
        size_t cap = 16;
        while (cap < (size_t)(2 * cnt + 16)) cap <<= 1;
        std::vector<int64_t> slot(cap, -1);
        int64_t d = 0;
        for (int64_t r = 0; r < n; ++r) {
            const uint64_t hr = h[(size_t)r];
            if ((int)(hr % (uint64_t)P) != part) continue;
            const int64_t a = rd(r), Lr = offsets[a + 1] - offsets[a];
            for (size_t s = (size_t)(hr >> 24) & (cap - 1);; s = (s + 1) & (cap - 1)) {
                const int64_t q = slot[s];
                if (q < 0) {
                    slot[s] = r;
                    rep[r] = r;
                    ++d;
                    break;
                }
                const int64_t b = rd(q);
                if (h[(size_t)q] == hr && offsets[b + 1] - offsets[b] == Lr &&
                    std::memcmp(reads + offsets[b], reads + offsets[a], (size_t)Lr) == 0) {
                    rep[r] = q;
                    break;
                }
            }
        }
        distinct[(size_t)part] = d;
    });
    int64_t tot = 0;
    for (int64_t d : distinct) tot += d;
    return tot;
}

extern "C" int nw_expand_ops(const char* ref, int32_t ref_len, const char* reads, const int64_t* offsets, int64_t n,
                             const uint32_t* ops, const int64_t* ops_off, char* aln_out, int64_t stride,
                             int32_t nthreads) {
    if (n < 0 || ref_len <= 0 || !ref || (n > 0 && (!reads || !offsets || !ops_off || !aln_out))) return NW_E_INVALID;
    const Tables& T = tables();
    std::vector<uint8_t> acode((size_t)ref_len);
    for (int32_t i = 0; i < ref_len; ++i) acode[(size_t)i] = T.code[(unsigned char)ref[i]];
    int nt = nthreads > 0 ? nthreads : nw_host::default_threads();
    nt = (int)std::max<int64_t>(1, std::min<int64_t>(nt, n / 4096 + 1));
    std::atomic<int> bad{0};
    auto work = [&](int64_t lo, int64_t hi) {
        for (int64_t r = lo; r < hi; ++r) {
            const int64_t Lb = offsets[r + 1] - offsets[r];
            const int64_t k0 = ops_off[r], k1 = ops_off[r + 1];
            if (Lb == 0 && k1 == k0) continue;   // empty read: no alignment
            if (k1 < k0 || !ops ||
                !expand_one(T, (const unsigned char*)ref, ref_len, acode.data(),
                            (const unsigned char*)reads + offsets[r], Lb, ops + k0, k1 - k0, aln_out + r * 3 * stride,
                            stride))
                bad.store(1, std::memory_order_relaxed);
        }
    };
    if (nt == 1) {
        work(0, n);
    } else {
        std::vector<std::thread> pool;
        const int64_t per = (n + nt - 1) / nt;
        for (int t = 0; t < nt; ++t) {
            const int64_t lo = t * per, hi = std::min(n, lo + per);
            if (lo < hi) pool.emplace_back(work, lo, hi);
        }
        for (auto& th : pool) th.join();
    }
    return bad.load() ? NW_E_INVALID : NW_OK;
}
