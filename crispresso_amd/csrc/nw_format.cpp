// nw_format.cpp -- srspair writer for GPU alignment records.
//
// Emits the blocks EMBOSS needle writes with -aformat srspair (its default) so
// that the reference parser parse_needle_output (CRISPRessoCORE.py:1707-1786)
// and the --keep_intermediate / --dump files (CRISPRessoCORE.py:3694-3697)
// keep working.  The parser depends on: the "# Aligned_sequences" marker, the
// read id as the last token of the "# 2:" line (:1724-1725), the identity as
// the last token of the "# Identity:" line (:1730-1738), seven skipped lines,
// then three alignment lines whose sequence column starts at byte 21
// (:1747-1754).
#include <cstdio>
#include <cstring>
#include <string>

#include "../../include/crispr_nw.h"

namespace {

struct Out {
    char* buf;
    int64_t cap;
    int64_t len = 0;
    void put(const char* s, int64_t n) {
        if (len + n <= cap) std::memcpy(buf + len, s, (size_t)n);
        len += n;
    }
    void puts(const char* s) { put(s, (int64_t)std::strlen(s)); }
    template <class... A>
    void printf(const char* fmt, A... a) {
        char tmp[512];
        int n = std::snprintf(tmp, sizeof tmp, fmt, a...);
        put(tmp, n);
    }
};

void name_field(Out& o, const char* name) {
    // %-13.13s
    char tmp[16];
    std::snprintf(tmp, sizeof tmp, "%-13.13s", name);
    o.put(tmp, 13);
}

}  // namespace

extern "C" int64_t nw_format_srspair(char* buf, int64_t cap, const char* aname, const char* bnames,
                                     float gap_open, float gap_extend, int32_t scale, int32_t awidth,
                                     const char* aln, int64_t stride, const nw_stat* stats, int64_t n) {
    Out o{buf, cap};
    if (awidth <= 0) awidth = 50;
    const char* bn = bnames;
    for (int64_t r = 0; r < n; ++r) {
        const char* bname = bn;
        bn += std::strlen(bn) + 1;
        const nw_stat& s = stats[r];
        if (s.flags & NW_FLAG_EMPTY) continue;
        const int32_t L = s.aln_len;
        const char* ra = aln + r * 3 * stride;
        const char* mk = ra + stride;
        const char* rb = mk + stride;
        const double pi = L ? 100.0 * s.n_ident / L : 0.0;
        const double ps = L ? 100.0 * s.n_sim / L : 0.0;
        const double pg = L ? 100.0 * s.n_gaps / L : 0.0;
        o.puts("#=======================================\n#\n# Aligned_sequences: 2\n# 1: ");
        o.puts(aname);
        o.puts("\n# 2: ");
        o.puts(bname);
        o.printf("\n# Matrix: EDNAFULL\n# Gap_penalty: %.1f\n# Extend_penalty: %.1f\n#\n", (double)gap_open,
                 (double)gap_extend);
        o.printf("# Length: %d\n", L);
        o.printf("# Identity:    %7d/%d (%4.1f%%)\n", s.n_ident, L, pi);
        o.printf("# Similarity:  %7d/%d (%4.1f%%)\n", s.n_sim, L, ps);
        o.printf("# Gaps:        %7d/%d (%4.1f%%)\n", s.n_gaps, L, pg);
        o.printf("# Score: %.1f\n# \n#\n#=======================================\n\n", (double)s.score / scale);
        int32_t na = 0, nb = 0;
        for (int32_t c0 = 0; c0 < L; c0 += awidth) {
            const int32_t w = (L - c0) < awidth ? (L - c0) : awidth;
            int32_t ca = 0, cb = 0;
            for (int32_t q = 0; q < w; ++q) {
                ca += ra[c0 + q] != '-';
                cb += rb[c0 + q] != '-';
            }
            if (c0) o.puts("\n");
            name_field(o, aname);
            o.printf(" %6d ", ca ? na + 1 : na);
            o.put(ra + c0, w);
            o.printf(" %6d\n", na + ca);
            o.printf("%21s", "");
            o.put(mk + c0, w);
            o.puts("\n");
            name_field(o, bname);
            o.printf(" %6d ", cb ? nb + 1 : nb);
            o.put(rb + c0, w);
            o.printf(" %6d\n", nb + cb);
            na += ca;
            nb += cb;
        }
        o.puts("\n\n");
    }
    if (o.len < cap) buf[o.len] = 0;
    return o.len;
}
