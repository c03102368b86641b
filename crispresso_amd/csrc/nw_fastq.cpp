// nw_fastq.cpp -- native FASTQ(.gz) ingest: the reads the reference's shell stage
// hands to needle (CRISPRessoCORE.py:1791-1797)
//
//     cat F | gunzip | awk 'NR % 4 == 1 {print ">" $0} NR % 4 == 2 {print $0}' | sed 's/:/_/g'
//
// as EMBOSS's FASTA reader then keeps them: the record name is the first
// whitespace-delimited word of the header line (':' already '_'), and the sequence
// keeps ASCII letters and the characters * . ~ ? # + - (so a ':' -- '_' after sed --
// and everything else is dropped).  Line 4k is a header, 4k + 1 its sequence; a
// header without a sequence line gives an empty read (awk still prints it).  The
// Python restatement crispresso_amd/fastq.py:fastq_bytes_as_fasta is the reference
// the tests hold this to.
//
// One pass over the decompressed stream (zlib gzread: plain files read through as
// well), 64 MB at a time: headers -> names ('\n'-joined), sequence lines filtered
// straight into one packed buffer + offsets, quality lines skipped by memchr.
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/crispr_nw.h"

struct nw_fastq {
    std::vector<char> seqs;
    std::vector<int64_t> offsets{0};
    std::vector<char> names;   // record names joined by '\n'
    std::string err;
};

namespace {

struct Tables {
    bool keep[256];
    bool ws[256];
    Tables() {
        for (int c = 0; c < 256; ++c) {
            const bool alpha = (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z');
            keep[c] = alpha || std::strchr("*.~?#+-", c) != nullptr;
            ws[c] = c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\x0b' || c == '\x0c';
        }
        keep[0] = false;
    }
};

const Tables& tables() {
    static const Tables t;
    return t;
}

struct Parser {
    nw_fastq* q;
    const Tables& T = tables();
    int64_t line = 0;           // index of the line being read
    bool name_started = false, name_done = false;
    int64_t headers = 0, seq_lines = 0;

    void end_line() {
        const int k = (int)(line & 3);
        if (k == 0) {   // header: one record; every name ends with '\n'
            q->names.push_back('\n');
            ++headers;
        } else if (k == 1) {
            q->offsets.push_back((int64_t)q->seqs.size());
            ++seq_lines;
        }
        ++line;
        name_started = name_done = false;
    }
    // bytes [p, e) of the current line (no '\n'; a line may arrive in several pieces)
    void feed(const unsigned char* p, const unsigned char* e) {
        const int k = (int)(line & 3);
        if (k == 0) {   // the first whitespace-delimited word, ':' -> '_'
            for (; p < e && !name_done; ++p) {
                const unsigned char ch = *p;
                if (T.ws[ch]) {
                    name_done = name_started;
                    continue;
                }
                name_started = true;
                q->names.push_back(ch == ':' ? '_' : (char)ch);
            }
        } else if (k == 1) {   // the bytes EMBOSS keeps (':' became '_', which it drops)
            std::vector<char>& v = q->seqs;
            const size_t at = v.size();
            if (v.capacity() < at + (size_t)(e - p)) v.reserve(std::max(2 * v.capacity(), at + (size_t)(e - p)));
            v.resize(at + (size_t)(e - p));
            char* d = v.data() + at;
            for (; p < e; ++p) {   // branch-free: write every byte, advance past the kept ones
                *d = (char)*p;
                d += T.keep[*p];
            }
            v.resize((size_t)(d - v.data()));
        }
    }
};

}  // namespace

extern "C" {

int nw_fastq_read(const char* path, nw_fastq** out) {
    if (!path || !out) return NW_E_INVALID;
    *out = nullptr;
    gzFile f = gzopen(path, "rb");
    if (!f) return NW_E_INVALID;
    (void)gzbuffer(f, 1 << 20);
    nw_fastq* q = new nw_fastq();
    Parser ps{q};
    std::vector<unsigned char> buf((size_t)64 << 20);
    bool pending = false;   // bytes of an unterminated line seen
    for (;;) {
        const int got = gzread(f, buf.data(), (unsigned)buf.size());
        if (got < 0) {
            int errnum = 0;
            q->err = gzerror(f, &errnum);
            gzclose(f);
            delete q;
            return NW_E_INVALID;
        }
        if (got == 0) break;
        const unsigned char* p = buf.data();
        const unsigned char* e = p + got;
        while (p < e) {
            const unsigned char* nl = (const unsigned char*)std::memchr(p, '\n', (size_t)(e - p));
            if ((ps.line & 3) >= 2) {   // quality / '+' lines: skip to the end of the line
                if (!nl) {
                    pending = true;
                    p = e;
                    break;
                }
                ps.end_line();
                pending = false;
                p = nl + 1;
                continue;
            }
            ps.feed(p, nl ? nl : e);
            if (!nl) {
                pending = true;
                p = e;
                break;
            }
            ps.end_line();
            pending = false;
            p = nl + 1;
        }
    }
    gzclose(f);
    if (pending) ps.end_line();   // a last line without '\n' is a line
    // a trailing header without a sequence line is a record with an empty read
    while (ps.seq_lines < ps.headers) {
        q->offsets.push_back((int64_t)q->seqs.size());
        ++ps.seq_lines;
    }
    *out = q;
    return NW_OK;
}

int64_t nw_fastq_count(const nw_fastq* q) { return q ? (int64_t)q->offsets.size() - 1 : -1; }
const char* nw_fastq_seqs(const nw_fastq* q) { return q ? q->seqs.data() : nullptr; }
const int64_t* nw_fastq_offsets(const nw_fastq* q) { return q ? q->offsets.data() : nullptr; }
// record names, each followed by '\n'
const char* nw_fastq_names(const nw_fastq* q, int64_t* bytes) {
    if (!q) return nullptr;
    if (bytes) *bytes = (int64_t)q->names.size();
    return q->names.data();
}
void nw_fastq_free(nw_fastq* q) { delete q; }

}  // extern "C"
