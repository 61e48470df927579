"""CPU oracle for the KGE scoring path — TEST INFRASTRUCTURE ONLY (see kge_oracle.py header).

PARITY UNPINNED: the reference ships no golden vectors or tests for this path and its TF /
upstream-PyTorch code cannot run here; this package restates it op for op.
"""
