"""TEST INFRASTRUCTURE ONLY — CPU restatements used as parity checkers.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package. Nothing under my_depthsplat_amd/ imports it: the product path runs on the GPU
through libdsplat_hip.so and fails loudly without it.

  oracle.raster        ctypes wrapper of build/libdsr_oracle.so (dsr_oracle.cpp):
                       the 3DGS rasterizer restated (forward + backward), "parity unpinned"
                       against the reference's absent CUDA library
  oracle.cost_volume   torch-fp32 restatement of matching.py:24-90 + mv_unimatch.py:494-505,
                       pinned by tests/golden/cost_volume.npz (generated from the reference)
  oracle.adapter       torch-fp32 restatement of gaussian_adapter.py:49-102,
                       pinned by tests/golden/adapter.npz
"""
