"""Minimal stand-in for the third-party ``roma`` package (unpinned in the
reference requirements.txt:3; absent from this image).  Only the surface the
reference calls in renderformer/utils/transform.py:24-27 is restated:
``Rigid.from_homogeneous``, ``inverse``, ``__getitem__``, ``apply`` and
``linear_apply`` for a rigid transform x -> R x + t (roma's published
definition).  Used only by tests/golden/make_golden.py to import the reference.
"""
import torch


class Rigid:
    def __init__(self, linear, translation):
        self.linear = linear
        self.translation = translation

    @staticmethod
    def from_homogeneous(m):
        return Rigid(m[..., :3, :3], m[..., :3, 3])

    def inverse(self):
        rt = self.linear.transpose(-1, -2)
        return Rigid(rt, -(rt @ self.translation[..., None])[..., 0])

    def __getitem__(self, idx):
        return Rigid(self.linear[idx], self.translation[idx])

    def linear_apply(self, x):
        return (self.linear @ x[..., None])[..., 0]

    def apply(self, x):
        return self.linear_apply(x) + self.translation
