"""MI355X-native RenderFormer inference path (HIP/CDNA4 kernels behind a C-ABI).

Import surface mirrors the reference package (renderformer/__init__.py:1-4):
``RenderFormer`` and ``RenderFormerRenderingPipeline``.  The model classes load
``librfhip.so`` on first use and raise if it is missing — there is no CPU or
eager-PyTorch fallback for the compute path.
"""
from .config import RenderFormerConfig

__all__ = ["RenderFormerRenderingPipeline", "RenderFormer", "RenderFormerConfig"]


def __getattr__(name):
    if name == "RenderFormer":
        from .model import RenderFormer
        return RenderFormer
    if name == "RenderFormerRenderingPipeline":
        from .pipeline import RenderFormerRenderingPipeline
        return RenderFormerRenderingPipeline
    raise AttributeError(name)
