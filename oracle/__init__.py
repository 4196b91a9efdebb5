"""Test-infrastructure oracle (CPU restatement of the reference hot path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  It is a checker, never the product path.  See cmt_oracle.py
header for the parity status (unpinned w.r.t. reference outputs).
"""
