"""mae_clip_amd: MI355X-native (gfx950) CLIP+MAE ViT training hot path.

Drop-in for the reference's modules.ImageEncoder / TextEncoder /
ProjectionHead and CLIP.CLIPModel (ykojima4020/mae_clip CLIP.py, modules.py),
backed by hand-written HIP kernels in libmaeclip.so (include/maeclip.h).
"""
__version__ = "0.1.0"
