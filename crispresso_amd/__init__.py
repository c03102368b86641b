"""crispresso_amd -- MI355X-native batched global aligner for CRISPResso.

Replaces the EMBOSS ``needle`` shell-out of CRISPResso's single-amplicon
pipeline (``CRISPResso/CRISPRessoCORE.py:1788-2000``) with a HIP kernel behind a
C ABI (``include/crispr_nw.h``).  See DESIGN.md and INTEGRATION.md.
"""
__version__ = "0.1.0"
