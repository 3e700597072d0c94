"""Drop-in ``RenderFormerRenderingPipeline`` (renderformer/pipelines/rendering_pipeline.py:8-128).

Same constructor, ``from_pretrained``, ``device``, ``to``, ``render`` and
``__call__`` with the same argument names, shapes, dtypes and return value
``[bs, num_views, H, W, 3]`` float32 linear HDR.  Like the reference it
log-encodes the emission channels of ``texture`` **in place**
(rendering_pipeline.py:67-68).

Precision: the reference GPU path switches stage precision with
``torch_dtype`` (rendering_pipeline.py:98-99, view_transformer.py:119: half ->
stage 1 half, stage 2 fp32, DPT half; fp32 -> stage 1 fp32, stage 2 bf16).  This
path runs ONE policy for every ``torch_dtype``: fp16 projection operands (bf16 with
``operands="bf16"``, or after an fp16 overflow: ``RenderFormer.range_check``), bf16
attention q/k/v, fp32 accumulation / softmax / residual streams in both transformer
stages, and fp16-operand, fp32-accumulate DPT convolutions — the policy measured
within the 1e-3 relative-L2 parity budget of the reference CPU fp32 output at every
BASELINE configuration (tests/test_parity_gpu.py).  The argument is validated
exactly like the reference; ``torch.float32`` (which in the reference selects
fp32 stage-1 arithmetic) emits a one-time ``PrecisionWarning`` saying so, and
``last_precision`` records what ran (``RenderFormer.precision``).

fp16 range check: by default (``RenderFormer(range_check="sync")``) ``render`` waits for its own
frame's end event — no device sync, the wait the caller's ``.cpu()`` would do anyway — and
re-renders an overflowed frame with bf16 operands before returning, so unchanged callers of the
reference API (README example, ``infer.py``) never see a non-finite frame.  Pipelining callers
(``batch_infer.py``) opt in to ``range_check="lazy"`` and call ``resolve(out)`` / ``check_range()``.
"""
from __future__ import annotations

import warnings

import torch

from .model import PrecisionWarning, RenderFormer  # noqa: F401  (PrecisionWarning re-exported)


class RenderFormerRenderingPipeline:
    def __init__(self, model: RenderFormer):
        self.model = model
        self.config = model.config
        self.last_precision = None
        self._warned_fp32 = False

    @classmethod
    def from_pretrained(cls, model_id: str, **kwargs):
        model = RenderFormer.from_pretrained(model_id, **kwargs)
        model.eval()
        return cls(model)

    @property
    def device(self):
        return self.model.device

    def to(self, device):
        self.model.to(device)
        return self

    def render(self, triangles, texture, mask, vn, c2w, fov, resolution: int = 512,
               torch_dtype: torch.dtype = torch.float16):
        """Render [bs, nv, resolution, resolution, 3] HDR images (rendering_pipeline.py:28-125)."""
        assert torch_dtype in [torch.bfloat16, torch.float16, torch.float32], (
            f"Invalid precision: {torch_dtype}\nChoose from: torch.bfloat16, torch.float16, torch.float32")
        if torch_dtype == torch.float32 and not self._warned_fp32:
            self._warned_fp32 = True
            warnings.warn("torch_dtype=torch.float32: this MI355X path has no fp32-operand mode; it computes with "
                          f"{self.model.precision} (within 1e-3 relative L2 of the reference's CPU fp32 output)",
                          PrecisionWarning, stacklevel=2)
        cfg = self.config
        if cfg.texture_encode_patch_size == 1 and texture.dim() == 5:
            texture = texture[:, :, :, 0, 0].contiguous()
        if not texture.is_contiguous():
            raise ValueError("texture must be contiguous (it is log-encoded in place)")
        if texture.dtype != torch.float32:
            raise ValueError("texture must be float32 (it is log-encoded in place)")
        out = self.model.render_views(triangles, texture, mask, vn, c2w, fov, resolution, log_encode=not cfg.use_ldr)
        self.last_precision = {"requested": str(torch_dtype), "computed": self.model.precision}
        return out

    def resolve(self, out=None) -> bool:
        """RenderFormer.resolve: finish the fp16 range check of the frame ``out`` (every pending frame if None),
        waiting for it; an overflowed frame is rendered again in place.  Only needed with range_check="lazy" (the
        default "sync" render has resolved its frame already; then this only reports whether it was re-rendered)."""
        redo = self.model.resolve(out)
        if self.last_precision is not None:
            self.last_precision["computed"] = self.model.precision
        return redo

    def check_range(self):
        """RenderFormer.check_range: resolve every pending frame (deferred mode: raise DeviceError if one
        overflowed; lazy: re-render it in place)."""
        try:
            self.model.check_range()
        finally:
            if self.last_precision is not None:
                self.last_precision["computed"] = self.model.precision

    def __call__(self, *args, **kwargs):
        return self.render(*args, **kwargs)
