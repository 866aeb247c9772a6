"""Parity oracle -- TEST INFRASTRUCTURE ONLY (see ref_model.py header).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
