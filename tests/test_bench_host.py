"""bench.py's host-side pieces (no GPU): the PMC traffic it reports comes from the
newest committed rocprofv3 summary under profiles/ and covers the band path's kernels."""
import importlib.util
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)   # module level: imports and constants only
    return mod


def test_pmc_summaries_exist_and_newest_first():
    b = load_bench()
    assert os.path.exists(b.PMC_SUMMARIES[0])
    with open(b.PMC_SUMMARIES[0]) as f:
        summ = json.load(f)
    assert any("nw_band_fill<16>" in k for k in summ)
    assert any("nw_band_walk<16>" in k for k in summ)


def test_band_traffic_from_committed_profile():
    b = load_bench()
    traffic, src = b.pmc_traffic("void nw::nw_band_", "nw::nw_band_", "void nw::nw_align_kernel",
                                 required="nw::nw_band_fill<16>")
    assert traffic is not None and traffic > 1e9   # ~3.3 GB per 1M C2 reads
    assert src == os.path.relpath(b.PMC_SUMMARIES[0], ROOT)


def test_quant_traffic_available():
    b = load_bench()
    traffic, _ = b.pmc_traffic("nwq::quant_kernel", "nwq::quant_reduce")
    assert traffic is not None and traffic > 0
