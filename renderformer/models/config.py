"""renderformer/models/config.py:5 — the hyper-parameter dataclass (same field names and defaults)."""
from renderformer_amd.config import RenderFormerConfig

__all__ = ["RenderFormerConfig"]
