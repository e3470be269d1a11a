"""ORACLE — CPU restatements of the reference arithmetic (test infrastructure).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / CPU baseline — never as the
product path.  See oracle/gravity_ref.c (C restatement of crates/gravity)
and oracle/profile_ref.py (numpy restatement of pynbodyext/profiles).
"""
