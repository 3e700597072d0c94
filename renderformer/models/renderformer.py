"""renderformer/models/renderformer.py:13 — the model (renderformer_amd.model)."""
from renderformer_amd.model import RenderFormer

__all__ = ["RenderFormer"]
