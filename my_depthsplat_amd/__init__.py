"""my_depthsplat_amd — MI355X-native hot path of yuehuarulian/my_depthsplat.

Differentiable 3D-Gaussian tile rasterizer + plane-sweep cost volume + Gaussian adapter,
hand-written HIP for gfx950 behind a C ABI (include/dsplat_hip.h), exposed through the
reference's own operator names:

  my_depthsplat_amd.rasterizer     GaussianRasterizationSettings, GaussianRasterizer
  my_depthsplat_amd.cuda_splatting render_cuda, render_depth_cuda, render_cuda_orthographic,
                                   get_projection_matrix (+ batched render_views)
  my_depthsplat_amd.decoder        Decoder, DecoderOutput, DecoderSplattingCUDA, DECODERS, get_decoder
  my_depthsplat_amd.matching       warp_with_pose_depth_candidates, plane_sweep_cost_volume
  my_depthsplat_amd.gaussian_adapter  GaussianAdapter, GaussianAdapterCfg
"""
__version__ = "0.1.0"
