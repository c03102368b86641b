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
// One pass over the decompressed stream: headers -> names ('\n'-joined), sequence
// lines filtered straight into one packed buffer + offsets, quality lines skipped by
// memchr.  Decompression: libdeflate when the image has it (dlopen'd libdeflate.so.0,
// whole gzip members into one buffer: ~7x zlib's inflate rate, 2.08 -> 0.29 s for the
// 1M-read C2 file on this container's CPU), else zlib gzread 64 MB at a time (also the
// path for files past kWholeMax, and CRISPR_NW_FASTQ_ZLIB=1).  Plain files go through
// either.
//
// Optional read quality filter (nw_fastq_read_filtered), the one CRISPResso applies
// before anything else when --min_average_read_quality / --min_single_bp_quality are
// set (filter_se_fastq_by_qual, CRISPRessoCORE.py:270-308, called at 1547-1583): a
// record is kept when the mean of its Phred+33 qualities is >= min_avg and their
// minimum >= min_single (integer test sum >= min_avg * n: exact, as numpy's float mean
// of integers is here); a record with an empty quality line is dropped (its numpy mean
// is NaN).  A dropped record's name and bases are rolled back.  pass[] keeps every
// record's verdict for the paired-end filter (by read id, in Python).
//
// nw_fastq_pack: the same reads as the aligner's packed input (nw_align_ops_packed: 2 bits
// per base + exception list) and a copy of the offsets, in page-locked memory, built once
// in parallel right after the parse -- what crosses PCIe (a quarter of the text's bytes)
// is ready in pinned buffers when ingest returns; the text stays for the rows
// (nw_expand_ops / the DataFrame hand-off).
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>
#include <zlib.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/crispr_nw.h"
#include "gz_inflate.h"
#include "host_pool.h"

// std::vector storage that resize() leaves uninitialised: the ingest's buffers are written
// in full right after they grow (a zero-fill of the 1M-read text alone was ~0.1 s).
template <class T>
struct NoInit : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInit<U>;
    };
    NoInit() = default;
    template <class U>
    NoInit(const NoInit<U>&) noexcept {}
    template <class U>
    void construct(U* p) noexcept {
        ::new ((void*)p) U;
    }
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        ::new ((void*)p) U(std::forward<A>(a)...);
    }
};

struct nw_fastq {
    std::vector<char, NoInit<char>> seqs;
    std::vector<int64_t, NoInit<int64_t>> offsets{0};
    std::vector<char, NoInit<char>> names;   // record names joined by '\n'
    std::vector<uint8_t> pass; // quality verdict of every record read (filtered reads only)
    int64_t dropped = 0;
    std::string err;
    // nw_fastq_pack: packed bases, offsets copy, exceptions (pinned or malloc'd)
    bool packed_done = false, packed_pinned = false;
    uint8_t* pk = nullptr;
    int64_t* pk_off = nullptr;
    int64_t* exc_pos = nullptr;
    uint8_t* exc_byte = nullptr;
    int64_t n_exc = 0;
    uint16_t* lens = nullptr;   // nw_fastq_lens (null: a read longer than 65535)
    void* blocks[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    ~nw_fastq() {
        for (void* b : blocks)
            if (b) {
                if (packed_pinned) (void)hipHostFree(b);
                else std::free(b);
            }
    }
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
    const Tables* T = &tables();
    int64_t line = 0;           // index of the line being read
    bool name_started = false, name_done = false;
    int64_t headers = 0, seq_lines = 0;
    // quality filter (filter = false: quality lines are skipped unread)
    bool filter = false;
    int64_t min_avg = 0, min_single = 0;
    int64_t qsum = 0, qn = 0, qmin = 1 << 30;
    size_t name_mark = 0;       // names.size() before the current record

    void end_line() {
        const int k = (int)(line & 3);
        if (k == 0) {   // header: one record; every name ends with '\n'
            q->names.push_back('\n');
            ++headers;
        } else if (k == 1) {
            q->offsets.push_back((int64_t)q->seqs.size());
            ++seq_lines;
        } else if (k == 3 && filter) {
            end_record();
        }
        ++line;
        name_started = name_done = false;
    }
    // the record's quality verdict; a failing record is taken back out
    void end_record() {
        const bool keep = qn > 0 && qsum >= min_avg * qn && qmin >= min_single;
        q->pass.push_back((uint8_t)keep);
        if (!keep) {
            q->names.resize(name_mark);
            q->offsets.pop_back();
            q->seqs.resize((size_t)q->offsets.back());
            --headers;
            --seq_lines;
            ++q->dropped;
        }
        name_mark = q->names.size();
        qsum = qn = 0;
        qmin = 1 << 30;
    }
    void feed_quality(const unsigned char* p, const unsigned char* e) {
        for (; p < e; ++p) {
            if (*p == '\r') continue;
            const int64_t v = (int64_t)*p - 33;
            qsum += v;
            qmin = v < qmin ? v : qmin;
            ++qn;
        }
    }
    // bytes [p, e) of the current line (no '\n'; a line may arrive in several pieces)
    void feed(const unsigned char* p, const unsigned char* e) {
        const int k = (int)(line & 3);
        if (k == 0) {   // the first whitespace-delimited word, ':' -> '_'
            for (; p < e && !name_done; ++p) {
                const unsigned char ch = *p;
                if (T->ws[ch]) {
                    name_done = name_started;
                    continue;
                }
                name_started = true;
                q->names.push_back(ch == ':' ? '_' : (char)ch);
            }
        } else if (k == 1) {   // the bytes EMBOSS keeps (':' became '_', which it drops)
            auto& v = q->seqs;
            const size_t at = v.size();
            if (v.capacity() < at + (size_t)(e - p)) v.reserve(std::max(2 * v.capacity(), at + (size_t)(e - p)));
            v.resize(at + (size_t)(e - p));
            char* d = v.data() + at;
            for (; p < e; ++p) {   // branch-free: write every byte, advance past the kept ones
                *d = (char)*p;
                d += T->keep[*p];
            }
            v.resize((size_t)(d - v.data()));
        }
    }
};

// decompressed bytes [p, e) of the stream; *pending: an unterminated line is open
void parse_block(Parser& ps, const unsigned char* p, const unsigned char* e, bool* pending) {
    while (p < e) {
        const unsigned char* nl = (const unsigned char*)std::memchr(p, '\n', (size_t)(e - p));
        if ((ps.line & 3) == 3 && ps.filter) ps.feed_quality(p, nl ? nl : e);
        if ((ps.line & 3) >= 2) {   // quality / '+' lines: skip to the end of the line
            if (!nl) {
                *pending = true;
                return;
            }
            ps.end_line();
            *pending = false;
            p = nl + 1;
            continue;
        }
        ps.feed(p, nl ? nl : e);
        if (!nl) {
            *pending = true;
            return;
        }
        ps.end_line();
        *pending = false;
        p = nl + 1;
    }
}

// libdeflate's whole-buffer gzip API (libdeflate.h 1.x), resolved at run time
struct Deflate {
    void* (*alloc)() = nullptr;
    int (*gzip_ex)(void*, const void*, size_t, void*, size_t, size_t*, size_t*) = nullptr;
    void (*release)(void*) = nullptr;
    uint32_t (*crc32)(uint32_t, const void*, size_t) = nullptr;   // optional (folding CRC)
    Deflate() {
        void* h = dlopen("libdeflate.so.0", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        alloc = (void* (*)())dlsym(h, "libdeflate_alloc_decompressor");
        gzip_ex = (int (*)(void*, const void*, size_t, void*, size_t, size_t*, size_t*))dlsym(
            h, "libdeflate_gzip_decompress_ex");
        release = (void (*)(void*))dlsym(h, "libdeflate_free_decompressor");
        crc32 = (uint32_t(*)(uint32_t, const void*, size_t))dlsym(h, "libdeflate_crc32");
        if (!alloc || !gzip_ex || !release) alloc = nullptr;
    }
    bool ok() const { return alloc != nullptr; }
};

const Deflate& deflate_lib() {
    static const Deflate d;
    return d;
}

constexpr size_t kWholeMax = (size_t)16 << 30;   // decompressed bytes held at once by the fast path
constexpr size_t kParallelMin = (size_t)16 << 20;  // smaller streams parse on one thread

// An anonymous mapping (huge pages where the kernel gives them): a buffer the size of a
// decompressed file without a zero-fill pass and with few page faults.
struct Mapping {
    unsigned char* p = nullptr;
    size_t n = 0;
    bool anon = false;
    ~Mapping() { release(); }
    void release() {
        if (p) munmap(p, n);
        p = nullptr;
        n = 0;
    }
    bool make(size_t bytes) {
        void* m = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
        if (m == MAP_FAILED) return false;
        (void)madvise(m, bytes, MADV_HUGEPAGE);
        p = (unsigned char*)m;
        n = bytes;
        anon = true;
        return true;
    }
    bool map_file(const char* path) {
        const int fd = open(path, O_RDONLY);
        if (fd < 0) return false;
        struct stat st;
        bool ok = fstat(fd, &st) == 0 && S_ISREG(st.st_mode) && st.st_size > 0 && (size_t)st.st_size <= kWholeMax;
        if (ok) {
            void* m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
            ok = m != MAP_FAILED;
            if (ok) {
                (void)madvise(m, (size_t)st.st_size, MADV_SEQUENTIAL | MADV_WILLNEED);
                p = (unsigned char*)m;
                n = (size_t)st.st_size;
            }
        }
        close(fd);
        return ok;
    }
};

// Copies the parser state that follows a record boundary: a part parsed on its own
// starts at line 0 of a record with an empty name mark.
void continue_from(Parser& ps, const Parser& part, int64_t lines_before, size_t names_before, int64_t headers,
                   int64_t seq_lines) {
    ps.line = lines_before + part.line;
    ps.name_started = part.name_started;
    ps.name_done = part.name_done;
    ps.headers = headers;
    ps.seq_lines = seq_lines;
    ps.qsum = part.qsum;
    ps.qn = part.qn;
    ps.qmin = part.qmin;
    ps.name_mark = names_before + part.name_mark;
}

// Bytes [b, b + len) of the stream into ps (which has seen nothing yet): cut into parts at
// record boundaries -- every part starts at a line whose index is 0 mod 4, known from a
// parallel newline count -- parsed in parallel into their own buffers, then joined.
void parse_parallel(Parser& ps, const unsigned char* b, size_t len, bool* pending) {
    nw_host::Pool& pool = nw_host::Pool::get();
    size_t par_min = kParallelMin;
    if (const char* e = std::getenv("CRISPR_NW_FASTQ_PAR_MIN")) par_min = (size_t)std::max(1ll, std::atoll(e));   // tests
    const int P = len < par_min ? 1 : pool.threads();
    if (P <= 1) {
        parse_block(ps, b, b + len, pending);
        return;
    }
    // newlines per raw slice
    std::vector<int64_t> nl((size_t)P, 0);
    pool.run(P, [&](int k) {
        int64_t lo, hi;
        nw_host::Pool::range((int64_t)len, P, k, &lo, &hi);
        int64_t c = 0;
        for (const unsigned char* x = b + lo; x < b + hi;) {
            const unsigned char* y = (const unsigned char*)std::memchr(x, '\n', (size_t)(b + hi - x));
            if (!y) break;
            ++c;
            x = y + 1;
        }
        nl[(size_t)k] = c;
    });
    // cut k: the first line start at or after slice k's start whose index is 0 mod 4
    std::vector<size_t> cut((size_t)P + 1, 0);
    std::vector<int64_t> line_at((size_t)P + 1, 0);
    int64_t before = 0;
    for (int k = 1; k <= P; ++k) {
        before += nl[(size_t)k - 1];
        if (k == P) {
            cut[(size_t)k] = len;
            continue;
        }
        int64_t lo, hi;
        nw_host::Pool::range((int64_t)len, P, k, &lo, &hi);
        size_t pos = (size_t)lo;
        int64_t idx = before;   // newlines in [0, lo): the index of the line holding lo
        if (pos > 0 && b[pos - 1] != '\n') {   // inside a line: move past its end (a newline of slice k)
            const unsigned char* y = (const unsigned char*)std::memchr(b + pos, '\n', len - pos);
            pos = y ? (size_t)(y - b) + 1 : len;
            idx += y ? 1 : 0;
        }
        while (pos < len && (idx & 3) != 0) {
            const unsigned char* y = (const unsigned char*)std::memchr(b + pos, '\n', len - pos);
            pos = y ? (size_t)(y - b) + 1 : len;
            idx += y ? 1 : 0;
        }
        if (pos < cut[(size_t)k - 1]) pos = cut[(size_t)k - 1];   // (never: cuts only move forward)
        cut[(size_t)k] = pos;
        line_at[(size_t)k] = idx;
    }
    // parts [cut k, cut k+1): parsed on their own
    std::vector<nw_fastq> parts((size_t)P);
    std::vector<Parser> pp;
    pp.reserve((size_t)P);
    for (int k = 0; k < P; ++k) {
        // capacity for the part's worst case (untouched pages cost nothing): no regrowth copies
        const size_t bytes = cut[(size_t)k + 1] - cut[(size_t)k];
        parts[(size_t)k].seqs.reserve(bytes);
        parts[(size_t)k].names.reserve(bytes);
        parts[(size_t)k].offsets.reserve(bytes / 6 + 2);
        pp.push_back(Parser{&parts[(size_t)k]});
        pp.back().filter = ps.filter;
        pp.back().min_avg = ps.min_avg;
        pp.back().min_single = ps.min_single;
    }
    std::vector<char> pend((size_t)P, 0);
    pool.run(P, [&](int k) {
        bool pe = false;
        parse_block(pp[(size_t)k], b + cut[(size_t)k], b + cut[(size_t)k + 1], &pe);
        pend[(size_t)k] = pe;
    });
    // join: sizes first, then the copies in parallel
    nw_fastq* q = ps.q;
    std::vector<size_t> s0((size_t)P + 1, 0), n0((size_t)P + 1, 0), o0((size_t)P + 1, 0), p0((size_t)P + 1, 0);
    int64_t headers = 0, seq_lines = 0;
    for (int k = 0; k < P; ++k) {
        const nw_fastq& f = parts[(size_t)k];
        s0[(size_t)k + 1] = s0[(size_t)k] + f.seqs.size();
        n0[(size_t)k + 1] = n0[(size_t)k] + f.names.size();
        o0[(size_t)k + 1] = o0[(size_t)k] + (f.offsets.size() - 1);
        p0[(size_t)k + 1] = p0[(size_t)k] + f.pass.size();
        q->dropped += f.dropped;
        headers += pp[(size_t)k].headers;
        seq_lines += pp[(size_t)k].seq_lines;
    }
    q->seqs.resize(s0[(size_t)P]);
    q->names.resize(n0[(size_t)P]);
    q->offsets.resize(1 + o0[(size_t)P]);
    q->pass.resize(p0[(size_t)P]);
    pool.run(P, [&](int k) {
        const nw_fastq& f = parts[(size_t)k];
        if (!f.seqs.empty()) std::memcpy(q->seqs.data() + s0[(size_t)k], f.seqs.data(), f.seqs.size());
        if (!f.names.empty()) std::memcpy(q->names.data() + n0[(size_t)k], f.names.data(), f.names.size());
        if (!f.pass.empty()) std::memcpy(q->pass.data() + p0[(size_t)k], f.pass.data(), f.pass.size());
        int64_t* o = q->offsets.data() + 1 + o0[(size_t)k];
        const int64_t base = (int64_t)s0[(size_t)k];
        for (size_t r = 1; r < f.offsets.size(); ++r) o[r - 1] = base + f.offsets[r];
    });
    // the last non-empty part's open state (an unfinished record or line) continues in ps
    int lastk = -1;
    for (int k = 0; k < P; ++k)
        if (cut[(size_t)k] < cut[(size_t)k + 1]) lastk = k;
    if (lastk < 0) return;
    continue_from(ps, pp[(size_t)lastk], line_at[(size_t)lastk], n0[(size_t)lastk], headers, seq_lines);
    *pending = pend[(size_t)lastk] != 0;
}

// The whole file (mapped), then every gzip member (or the plain bytes) into one buffer,
// parsed in parallel.  1: done; 0: not taken (no libdeflate, too big, not decodable here:
// the zlib path reads the file, and reports its errors); -1: failed part-way.
int read_whole(const char* path, Parser& ps, bool* pending) {
    const char* zl = std::getenv("CRISPR_NW_FASTQ_ZLIB");
    if (zl && std::strcmp(zl, "1") == 0) return 0;
    Mapping in;
    if (!in.map_file(path)) return 0;
    const bool gz = in.n >= 18 && in.p[0] == 0x1f && in.p[1] == 0x8b;
    if (!gz) {
        parse_parallel(ps, in.p, in.n, pending);
        return 1;
    }
    const Deflate& D = deflate_lib();
    {   // one member decoded by all the pool's threads (gz_inflate.h); else one thread below
        nw_gz::Buffer whole;
        if (nw_gz::inflate_parallel(in.p, in.n, nw_host::Pool::get().threads(), D.crc32, &whole)) {
            parse_parallel(ps, whole.p, whole.n, pending);
            whole.release();
            return 1;
        }
    }
    if (!D.ok()) return 0;
    void* dec = D.alloc();
    if (!dec) return 0;
    // the last member's ISIZE (uncompressed size mod 2^32) sizes the first attempt
    const size_t isize = (size_t)in.p[in.n - 4] | (size_t)in.p[in.n - 3] << 8 | (size_t)in.p[in.n - 2] << 16 |
                         (size_t)in.p[in.n - 1] << 24;
    size_t pos = 0, cap = std::max(isize, 4 * in.n) + 4096;
    nw_host::Pool& pool = nw_host::Pool::get();
    int rc = 1;
    bool first = true;
    while (pos + 18 <= in.n && in.p[pos] == 0x1f && in.p[pos + 1] == 0x8b) {
        Mapping outb;
        size_t ain = 0, aout = 0;
        int r = 3;
        for (;;) {   // LIBDEFLATE_INSUFFICIENT_SPACE (3): a bigger buffer, same member
            if (!outb.make(cap)) break;
            if (cap >= kParallelMin) {   // the page faults of the output, taken in parallel before the serial inflate
                const int P = pool.threads();
                const size_t touch = std::min(cap, isize + 4096);
                pool.run(P, [&](int k) {
                    int64_t lo, hi;
                    nw_host::Pool::range((int64_t)touch, P, k, &lo, &hi);
                    for (int64_t b = lo & ~(int64_t)4095; b < hi; b += 4096) outb.p[b] = 0;
                });
            }
            r = D.gzip_ex(dec, in.p + pos, in.n - pos, outb.p, outb.n, &ain, &aout);
            if (r != 3 || cap >= kWholeMax) break;
            outb.release();
            cap = std::min(kWholeMax, 2 * cap);
        }
        if (r != 0 || ain == 0) {   // bad data (or a member past kWholeMax): the zlib path decides
            rc = first ? 0 : -1;
            break;
        }
        if (first && pos + ain >= in.n) parse_parallel(ps, outb.p, aout, pending);   // one member: the usual file
        else parse_block(ps, outb.p, outb.p + aout, pending);
        first = false;
        pos += ain;
    }
    D.release(dec);
    return rc;   // trailing bytes that are not a gzip member are ignored, as gzread does
}

}  // namespace

extern "C" {

int nw_fastq_read_filtered(const char* path, int32_t min_avg_quality, int32_t min_single_quality, nw_fastq** out) {
    if (!path || !out) return NW_E_INVALID;
    *out = nullptr;
    nw_fastq* q = new nw_fastq();
    Parser ps{q};
    ps.filter = min_avg_quality > 0 || min_single_quality > 0;
    ps.min_avg = min_avg_quality;
    ps.min_single = min_single_quality;
    bool pending = false;   // bytes of an unterminated line seen
    const int whole = read_whole(path, ps, &pending);
    if (whole < 0) {   // a later member failed after earlier ones were parsed: start over on zlib
        delete q;
        q = new nw_fastq();
        ps = Parser{q};
        ps.filter = min_avg_quality > 0 || min_single_quality > 0;
        ps.min_avg = min_avg_quality;
        ps.min_single = min_single_quality;
        pending = false;
    }
    if (whole <= 0) {
        gzFile f = gzopen(path, "rb");
        if (!f) {
            delete q;
            return NW_E_INVALID;
        }
        (void)gzbuffer(f, 1 << 20);
        std::vector<unsigned char> buf((size_t)64 << 20);
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
            parse_block(ps, buf.data(), buf.data() + got, &pending);
        }
        gzclose(f);
    }
    if (pending) ps.end_line();   // a last line without '\n' is a line
    // a trailing header without a sequence line is a record with an empty read
    while (ps.seq_lines < ps.headers) {
        q->offsets.push_back((int64_t)q->seqs.size());
        ++ps.seq_lines;
    }
    // a record cut off before its quality line: no qualities (mean NaN), dropped
    if (ps.filter && (ps.line & 3) != 0) ps.end_record();
    *out = q;
    return NW_OK;
}

int nw_fastq_read(const char* path, nw_fastq** out) { return nw_fastq_read_filtered(path, 0, 0, out); }

int64_t nw_fastq_dropped(const nw_fastq* q) { return q ? q->dropped : -1; }
// quality verdict of every record of the file (nw_fastq_read_filtered with a threshold)
const uint8_t* nw_fastq_pass(const nw_fastq* q, int64_t* n) {
    if (!q) return nullptr;
    if (n) *n = (int64_t)q->pass.size();
    return q->pass.data();
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

int nw_fastq_pack(nw_fastq* q, int32_t pinned, const uint8_t** packed, const int64_t** offsets, const int64_t** exc_pos,
                  const uint8_t** exc_byte, int64_t* n_exc) {
    if (!q) return NW_E_INVALID;
    if (q->packed_done && q->packed_pinned != (pinned != 0)) return NW_E_STATE;   // built the other way already
    if (!q->packed_done) {
        const int64_t n = (int64_t)q->offsets.size() - 1;
        const int64_t nb = q->offsets.back();
        auto get = [&](size_t bytes, int k) -> void* {
            bytes = std::max<size_t>(bytes, 64);
            void* p = nullptr;
            if (pinned) {
                if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) p = nullptr;
            } else {
                p = std::malloc(bytes);
            }
            q->blocks[k] = p;
            return p;
        };
        q->packed_pinned = pinned != 0;
        q->pk = (uint8_t*)get((size_t)(nb + 3) / 4 + 16, 0);
        q->pk_off = (int64_t*)get(sizeof(int64_t) * (size_t)(n + 1), 1);
        if (!q->pk || !q->pk_off) return NW_E_NOMEM;
        std::memcpy(q->pk_off, q->offsets.data(), sizeof(int64_t) * (size_t)(n + 1));
        // exceptions: N and other non-ACGT bytes, usually few; a second pass sizes a big list
        int64_t cap = nb / 64 + 4096, got = 0;
        std::vector<int64_t> pos((size_t)cap);
        std::vector<uint8_t> byt((size_t)cap);
        const int nt = nw_host::Pool::get().threads();
        int rc = nw_pack_reads(q->seqs.data(), q->offsets.data(), n, q->pk, pos.data(), byt.data(), cap, &got, nt);
        if (rc == NW_E_CAPACITY) {
            cap = got;
            pos.assign((size_t)cap, 0);
            byt.assign((size_t)cap, 0);
            rc = nw_pack_reads(q->seqs.data(), q->offsets.data(), n, q->pk, pos.data(), byt.data(), cap, &got, nt);
        }
        if (rc) return rc;
        q->exc_pos = (int64_t*)get(sizeof(int64_t) * (size_t)got, 2);
        q->exc_byte = (uint8_t*)get((size_t)got, 3);
        if (!q->exc_pos || !q->exc_byte) return NW_E_NOMEM;
        if (got) {
            std::memcpy(q->exc_pos, pos.data(), sizeof(int64_t) * (size_t)got);
            std::memcpy(q->exc_byte, byt.data(), (size_t)got);
        }
        q->n_exc = got;
        // the lengths (nw_align_ops_packed_lens: they cross PCIe instead of the offsets)
        q->lens = (uint16_t*)get(sizeof(uint16_t) * (size_t)std::max<int64_t>(n, 1), 4);
        if (!q->lens) return NW_E_NOMEM;
        if (nw_read_lengths16(q->offsets.data(), n, q->lens, nt) != NW_OK) q->lens = nullptr;
        q->packed_done = true;
    }
    if (packed) *packed = q->pk;
    if (offsets) *offsets = q->pk_off;
    if (exc_pos) *exc_pos = q->exc_pos;
    if (exc_byte) *exc_byte = q->exc_byte;
    if (n_exc) *n_exc = q->n_exc;
    return NW_OK;
}

// The ID column of parse_needle_output (CRISPRessoCORE.py:1725: the name line's last word with
// '_' back to ':') from names joined by '\n' (nw_fastq_names): ids = the bytes without the
// newlines, '_' -> ':'; off[i] .. off[i + 1] = name i.  NW_E_UNSUPPORTED when a name holds
// whitespace or a non-ASCII byte (then split() decides, in Python) or the newlines are not n.
int nw_names_to_ids(const uint8_t* raw, int64_t nbytes, int64_t n, uint8_t* ids, int64_t* off) {
    if (nbytes < 0 || n < 0 || (nbytes > 0 && (!raw || !ids)) || !off) return NW_E_INVALID;
    off[0] = 0;
    if (nbytes == 0) return n == 0 ? NW_OK : NW_E_UNSUPPORTED;
    nw_host::Pool& pool = nw_host::Pool::get();
    const int P = (int)std::max<int64_t>(1, std::min<int64_t>(pool.threads(), nbytes >> 20));
    std::vector<int64_t> nl((size_t)P + 1, 0);
    pool.run(P, [&](int k) {
        int64_t lo, hi, c = 0;
        nw_host::Pool::range(nbytes, P, k, &lo, &hi);
        for (int64_t p = lo; p < hi; ++p) c += raw[p] == '\n';
        nl[(size_t)k + 1] = c;
    });
    for (int k = 0; k < P; ++k) nl[(size_t)k + 1] += nl[(size_t)k];
    if (nl[(size_t)P] != n || raw[nbytes - 1] != '\n') return NW_E_UNSUPPORTED;
    std::vector<char> bad((size_t)P, 0);
    pool.run(P, [&](int k) {
        int64_t lo, hi, i = nl[(size_t)k];
        nw_host::Pool::range(nbytes, P, k, &lo, &hi);
        unsigned char acc = 0;
        bool ws = false;
        for (int64_t p = lo; p < hi; ++p) {
            const unsigned char ch = raw[p];
            if (ch == '\n') {
                off[i + 1] = p - i;   // name i ends here (i newlines before it)
                ++i;
                continue;
            }
            acc |= ch;
            ws |= ch == ' ' || ch == '\t' || ch == '\r' || ch == '\f' || ch == '\v' || (ch >= 0x1c && ch <= 0x1f);
            ids[p - i] = ch == '_' ? ':' : ch;
        }
        bad[(size_t)k] = (acc & 0x80) || ws;
    });
    for (char b : bad)
        if (b) return NW_E_UNSUPPORTED;
    return NW_OK;
}

// The ingest's parallel decompressor on its own (gz_inflate.h): the bytes of a one-member
// gzip image into out[0 .. cap).  NW_E_UNSUPPORTED when it does not take the image (the
// ingest then decodes on one thread), NW_E_CAPACITY when cap is short (*out_n = the size).
int nw_gunzip_parallel(const uint8_t* gz, int64_t n, int32_t threads, uint8_t* out, int64_t cap, int64_t* out_n) {
    if (!gz || n < 0 || !out_n || (cap > 0 && !out)) return NW_E_INVALID;
    nw_gz::Buffer b;
    if (!nw_gz::inflate_parallel(gz, (size_t)n, threads, deflate_lib().crc32, &b)) return NW_E_UNSUPPORTED;
    *out_n = (int64_t)b.n;
    const int rc = (int64_t)b.n > cap ? NW_E_CAPACITY : NW_OK;
    if (rc == NW_OK) std::memcpy(out, b.p, b.n);
    b.release();
    return rc;
}

int nw_fastq_lens(nw_fastq* q, const uint16_t** lens) {
    if (!q || !lens) return NW_E_INVALID;
    if (!q->packed_done) return NW_E_STATE;   // nw_fastq_pack first
    *lens = q->lens;
    return q->lens ? NW_OK : NW_E_UNSUPPORTED;
}

}  // extern "C"
