"""storb_amd — MI355X-native Reed–Solomon erasure coding for storb's chunk-and-shard path.

Layers:
  include/storb_ec.h, storb_amd/csrc/   C ABI + hand-written gfx950 HIP kernels (libstorbec.so)
  storb_amd._lib                        ctypes binding (fails loudly when the .so is missing)
  storb_amd.engine                      per-(device, thread) context, host and device batches
  storb_amd.easyfec                     zfec.easyfec-compatible Encoder / Decoder
  storb_amd.piece                       drop-in for storb/util/piece.py
  storb_amd.dist                        one-process-per-GPU chunk partitioning (no collective)
"""

__version__ = "0.1.0"
