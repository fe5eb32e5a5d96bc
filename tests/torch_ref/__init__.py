"""Test-only reference data plane: the workloads re-implemented in plain
PyTorch over torch.distributed point-to-point (halo exchange through
isend/irecv, fields as torch tensors).  The framework's data plane is the
native engine (csrc/engine, gpu_mpi_tests_amd/engine.py); these modules exist
only so the tests can cross-check it against an independent implementation
of the same decomposition and exchange semantics."""
