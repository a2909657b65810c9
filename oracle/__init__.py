"""ORACLE — CPU restatement of the reference hot path.  Test infrastructure only: imported by
tests/, __graft_entry__.smoke() (as the checker) and bench.py's cpu_baseline leg, never by the
product package textmae-image-compression_amd/."""
