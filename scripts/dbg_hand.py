import os, sys
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
from crispresso_amd.aligner import GpuAligner
from crispresso_amd.aligner import pack_reads
amp = "ACGTACGTTTGACCA"
sets = [["ACGTRYKMSWBDHVNU"], ["ACGTRYKMSWBDHVNU", "ACGTACGTTTGACCAGG"],
        ["ACGTACGTGACCA", "ACGTACGTTTGACCAGG", "TTGACC", "A", "ACGTACGTTTGACCA", "", "acgtNNNNtttgacca",
         "GGGGGGGGGGGGGGGGGGGGGGGGGGGGGG", "T-C-A", "ACGTRYKMSWBDHVNU"]]
for reads in sets:
    a = GpuAligner()
    a.set_reference(amp)
    buf, off = pack_reads(reads)
    b = a.align_packed(buf, off)
    print(len(reads), [int(x) for x in b.stats["score"]], a.fallbacks() if hasattr(a, "fallbacks") else "")
reads = sets[2]
buf, off = pack_reads(reads)
for rep in range(int(os.environ.get("REPS", "6"))):
    a = GpuAligner()
    a.set_reference(amp)
    b = a.align_packed(buf, off)
    print("rep", rep, int(b.stats["score"][9]), a.fallbacks())
    a.close()
