"""ORACLE — test infrastructure only (see oracle/csum_oracle.c header).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product (rustnetworkstack_amd) never does.
"""
