"""CPU oracle for the GAT hot path -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() (as the checker) and bench.py's
``cpu_baseline`` leg (as the timed CPU baseline).  Never by the product package.
See gat_oracle.py for what each function restates (reference file:line).
"""
