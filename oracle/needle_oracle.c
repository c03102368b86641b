/*
 * needle_oracle.c -- `needle`-compatible command line over the CPU oracle.
 *
 * TEST INFRASTRUCTURE ONLY: used to generate golden fixtures by running the
 * reference's own shell pipeline (CRISPRessoCORE.py:1791-1806) with this binary
 * standing in for EMBOSS needle, and as the CPU baseline in bench.py.
 *
 * Accepts the EMBOSS qualifier forms CRISPResso uses: -asequence=F
 * -bsequence=F -outfile=F -gapopen=X -gapextend=Y -awidth3=N (also "-q value").
 * FASTA input keeps letters and the gap/stop characters "*.~?#+-" as EMBOSS's
 * sequence reader does; the sequence name is the first word after '>'.
 */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <ctype.h>

#include "nw_oracle.h"

typedef struct { char* name; char* seq; int32_t len; } rec;

static int keep_char(int c) {
    return isalpha(c) || (c && strchr("*.~?#+-", c) != NULL);
}

/* Reads the next FASTA record; returns 0 at EOF. */
static int next_record(FILE* f, rec* r, char** pending) {
    size_t cap = 0; char* line = NULL; ssize_t n;
    char* hdr = *pending;
    *pending = NULL;
    while (!hdr) {
        n = getline(&line, &cap, f);
        if (n < 0) { free(line); return 0; }
        if (line[0] == '>') { hdr = strdup(line); }
    }
    /* name = first whitespace-delimited token after '>' */
    char* p = hdr + 1;
    while (*p && isspace((unsigned char)*p)) p++;
    char* e = p;
    while (*e && !isspace((unsigned char)*e)) e++;
    r->name = strndup(p, e - p);
    free(hdr);
    size_t scap = 256, slen = 0;
    r->seq = (char*)malloc(scap);
    while ((n = getline(&line, &cap, f)) >= 0) {
        if (line[0] == '>') { *pending = strdup(line); break; }
        for (ssize_t i = 0; i < n; i++) {
            int c = (unsigned char)line[i];
            if (!keep_char(c)) continue;
            if (slen + 1 >= scap) { scap *= 2; r->seq = (char*)realloc(r->seq, scap); }
            r->seq[slen++] = (char)c;
        }
    }
    r->seq[slen] = 0;
    r->len = (int32_t)slen;
    free(line);
    return 1;
}

static const char* opt_value(int argc, char** argv, int* i, const char* key) {
    size_t kl = strlen(key);
    const char* a = argv[*i];
    if (a[0] != '-') return NULL;
    a++;
    if (strncmp(a, key, kl) != 0) return NULL;
    if (a[kl] == '=') return a + kl + 1;
    if (a[kl] == 0 && *i + 1 < argc) { (*i)++; return argv[*i]; }
    return NULL;
}

int main(int argc, char** argv) {
    const char *afile = NULL, *bfile = NULL, *ofile = "stdout";
    float gapopen = 10.0f, gapextend = 0.5f, endopen = 10.0f, endextend = 0.5f;
    int endweight = 0;
    for (int i = 1; i < argc; i++) {
        const char* v;
        if (strcmp(argv[i], "-endweight") == 0) { endweight = 1; continue; }
        if (strcmp(argv[i], "-noendweight") == 0) { endweight = 0; continue; }
        if ((v = opt_value(argc, argv, &i, "asequence"))) afile = v;
        else if ((v = opt_value(argc, argv, &i, "bsequence"))) bfile = v;
        else if ((v = opt_value(argc, argv, &i, "outfile"))) ofile = v;
        else if ((v = opt_value(argc, argv, &i, "gapopen"))) gapopen = strtof(v, NULL);
        else if ((v = opt_value(argc, argv, &i, "gapextend"))) gapextend = strtof(v, NULL);
        else if ((v = opt_value(argc, argv, &i, "endopen"))) endopen = strtof(v, NULL);
        else if ((v = opt_value(argc, argv, &i, "endextend"))) endextend = strtof(v, NULL);
        else if ((v = opt_value(argc, argv, &i, "awidth3"))) (void)v;
        else if (strcmp(argv[i], "-auto") == 0 || strcmp(argv[i], "-stdout") == 0) continue;
        else { fprintf(stderr, "needle_oracle: unsupported option %s\n", argv[i]); return 1; }
    }
    if (!afile || !bfile) { fprintf(stderr, "needle_oracle: -asequence and -bsequence required\n"); return 1; }
    oracle_params P;
    if (oracle_params_init_end(&P, gapopen, gapextend, endweight, endopen, endextend)) {
        fprintf(stderr, "needle_oracle: penalties not representable\n");
        return 1;
    }
    FILE* fa = fopen(afile, "r");
    if (!fa) { fprintf(stderr, "needle_oracle: cannot open %s: %s\n", afile, strerror(errno)); return 1; }
    char* pend = NULL;
    rec A;
    if (!next_record(fa, &A, &pend) || A.len == 0) { fprintf(stderr, "needle_oracle: empty -asequence\n"); return 1; }
    fclose(fa); free(pend); pend = NULL;
    FILE* fb = strcmp(bfile, "/dev/stdin") == 0 || strcmp(bfile, "stdin") == 0 ? stdin : fopen(bfile, "r");
    if (!fb) { fprintf(stderr, "needle_oracle: cannot open %s\n", bfile); return 1; }
    FILE* fo = (strcmp(ofile, "/dev/stdout") == 0 || strcmp(ofile, "stdout") == 0) ? stdout : fopen(ofile, "w");
    if (!fo) { fprintf(stderr, "needle_oracle: cannot open %s\n", ofile); return 1; }
    fprintf(fo, "########################################\n# Program: needle\n# Rundate: (oracle)\n"
                "# Commandline: needle\n#    -asequence %s\n#    -bsequence %s\n"
                "# Align_format: srspair\n# Report_file: %s\n"
                "########################################\n\n", afile, bfile, ofile);
    rec B;
    size_t cap = 0; char *ra = NULL, *mk = NULL, *rb = NULL, *txt = NULL; size_t tcap = 0;
    while (next_record(fb, &B, &pend)) {
        if (B.len == 0) { free(B.name); free(B.seq); continue; }
        size_t need = (size_t)A.len + B.len + 1;
        if (need > cap) {
            cap = need * 2;
            ra = (char*)realloc(ra, cap); mk = (char*)realloc(mk, cap); rb = (char*)realloc(rb, cap);
        }
        oracle_result R;
        if (oracle_align(A.seq, A.len, B.seq, B.len, &P, &R, ra, mk, rb)) {
            fprintf(stderr, "needle_oracle: alignment failed\n");
            return 1;
        }
        int64_t n = oracle_format_srspair(txt, (int64_t)tcap, A.name, B.name, &P, &R, ra, mk, rb);
        if (n >= (int64_t)tcap) {
            tcap = (size_t)n * 2 + 1;
            txt = (char*)realloc(txt, tcap);
            n = oracle_format_srspair(txt, (int64_t)tcap, A.name, B.name, &P, &R, ra, mk, rb);
        }
        fwrite(txt, 1, (size_t)n, fo);
        free(B.name); free(B.seq);
    }
    fprintf(fo, "#---------------------------------------\n#---------------------------------------\n");
    if (fo != stdout) fclose(fo);
    return 0;
}
