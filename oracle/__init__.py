"""Test-only oracle for the EEGNet train/infer step (see numpy_ref.py / torch_ref.py headers).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
