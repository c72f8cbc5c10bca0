"""vfx_image_stitching_amd -- MI355X (gfx950) hot path of sapt36/VFX_Image_Stitching.

Drop-in modules mirroring the reference's function API:
  vfx_image_stitching_amd.sift_impl               <- sift_impl.py
  vfx_image_stitching_amd.image_stitching_sift    <- image_stitching_sift.py
  vfx_image_stitching_amd.image_stitching_harris  <- image_stitching_harris.py
Batched pipeline: vfx_image_stitching_amd.pipeline.Stitcher; multi-GPU: .distributed.
All compute goes through libpano.so (include/pano.h); there is no CPU fallback.
"""
from ._lib import PanoError, load  # noqa: F401

__version__ = "0.1.0"
