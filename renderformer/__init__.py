"""The reference's import surface (renderformer/__init__.py:1-4), served by the MI355X-native path.

``from renderformer import RenderFormerRenderingPipeline`` (README.md:155-187) and the reference's module
paths (``renderformer.pipelines.rendering_pipeline``, ``renderformer.models.renderformer``,
``renderformer.models.config``) resolve to ``renderformer_amd``: the HIP kernels behind librfhip.so, with no
CPU or eager-PyTorch fallback.
"""
from renderformer_amd.model import RenderFormer
from renderformer_amd.pipeline import RenderFormerRenderingPipeline

__all__ = ['RenderFormerRenderingPipeline', 'RenderFormer']
