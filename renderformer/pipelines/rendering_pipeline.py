"""renderformer/pipelines/rendering_pipeline.py:8 — the drop-in pipeline (renderformer_amd.pipeline)."""
from renderformer_amd.pipeline import RenderFormerRenderingPipeline

__all__ = ["RenderFormerRenderingPipeline"]
