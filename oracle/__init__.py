"""CPU oracle for the storb erasure-coding path — TEST INFRASTRUCTURE ONLY.

Parity status: **unpinned against real zfec bytes** (zfec 1.6.0.0 is absent from
/root/reference and this image; see fec_oracle.c header).  Importable only from
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
