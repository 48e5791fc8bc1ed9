"""Parameter initializers (``paddle.fluid.initializer`` surface).

Each initializer fills a torch tensor in place; the startup program records
one ``init_param`` op per parameter and the executor applies it
(reference: ``py/fluid/initializer.py``; fan-in/fan-out conventions follow
the fluid ``[in, out]`` fc weight layout).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def _fans(shape):
    if len(shape) == 0:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    rf = int(np.prod(shape[2:]))
    return shape[1] * rf, shape[0] * rf


class Initializer:
    def __call__(self, t: torch.Tensor, gen: torch.Generator):
        raise NotImplementedError


class ConstantInitializer(Initializer):
    def __init__(self, value=0.0, force_cpu=False):
        self.value = float(value)

    def __call__(self, t, gen):
        t.fill_(self.value)


class UniformInitializer(Initializer):
    def __init__(self, low=-1.0, high=1.0, seed=0, **_):
        self.low, self.high, self.seed = float(low), float(high), seed

    def __call__(self, t, gen):
        u = torch.rand(t.shape, generator=gen, dtype=torch.float32)
        t.copy_(u * (self.high - self.low) + self.low)


class NormalInitializer(Initializer):
    def __init__(self, loc=0.0, scale=1.0, seed=0):
        self.loc, self.scale, self.seed = float(loc), float(scale), seed

    def __call__(self, t, gen):
        t.copy_(torch.randn(t.shape, generator=gen) * self.scale + self.loc)


class TruncatedNormalInitializer(NormalInitializer):
    def __call__(self, t, gen):
        x = torch.randn(t.shape, generator=gen)
        bad = x.abs() > 2.0
        while bool(bad.any()):
            x[bad] = torch.randn(int(bad.sum()), generator=gen)
            bad = x.abs() > 2.0
        t.copy_(x * self.scale + self.loc)


class XavierInitializer(Initializer):
    def __init__(self, uniform=True, fan_in=None, fan_out=None, seed=0):
        self.uniform, self.fan_in, self.fan_out, self.seed = uniform, fan_in, fan_out, seed

    def __call__(self, t, gen):
        fi, fo = _fans(list(t.shape))
        fi = self.fan_in or fi
        fo = self.fan_out or fo
        if self.uniform:
            lim = math.sqrt(6.0 / (fi + fo))
            t.copy_(torch.rand(t.shape, generator=gen) * 2 * lim - lim)
        else:
            t.copy_(torch.randn(t.shape, generator=gen) * math.sqrt(2.0 / (fi + fo)))


class MSRAInitializer(Initializer):
    def __init__(self, uniform=True, fan_in=None, seed=0):
        self.uniform, self.fan_in, self.seed = uniform, fan_in, seed

    def __call__(self, t, gen):
        fi, _ = _fans(list(t.shape))
        fi = self.fan_in or fi
        if self.uniform:
            lim = math.sqrt(6.0 / fi)
            t.copy_(torch.rand(t.shape, generator=gen) * 2 * lim - lim)
        else:
            t.copy_(torch.randn(t.shape, generator=gen) * math.sqrt(2.0 / fi))


class NumpyArrayInitializer(Initializer):
    def __init__(self, value):
        self.value = np.asarray(value)

    def __call__(self, t, gen):
        t.copy_(torch.as_tensor(self.value).reshape(t.shape))


Constant = ConstantInitializer
Uniform = UniformInitializer
Normal = NormalInitializer
TruncatedNormal = TruncatedNormalInitializer
Xavier = XavierInitializer
MSRA = MSRAInitializer
