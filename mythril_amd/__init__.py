"""mythril_amd — MI355X-native batched path-constraint evaluator for Mythril's quick-sat path.

The hot path of the reference is ModelCache.check_quick_sat (mythril/support/support_utils.py:60-67)
reached from get_model (mythril/support/model.py:68-130).  This package provides:
  tape       — z3-independent constraint IR (the lowering target)
  models     — candidate-model batches (SoA u32 limbs + UF/array tables)
  evaluator  — ctypes binding of libmq.so (HIP kernels for gfx950, C-ABI include/mq.h)
  support    — drop-in mirrors of get_model / ModelCache / LRUCache backed by the GPU
  synth      — seeded synthetic workloads
"""
__version__ = "0.1.0"
