"""Channel plugins (reference core/channels.py:11-27,78-83,132-146).

``OkumuraHata`` is evaluated on the GPU: libmev builds the Okumura-Hata -> SNR -> Shannon
rate table over every integer squared distance when the engine is created and the step
kernel looks the serving pair up in it. Per-pair host evaluation is not provided (no CPU
path); subclasses with their own ``power_loss`` have no device lowering.
"""
from __future__ import annotations

EPSILON = 1e-16  # channels.py:8


class Channel:
    def __init__(self, **kwargs):
        pass

    def reset(self) -> None:
        pass

    def power_loss(self, bs, ue) -> float:
        raise NotImplementedError("channel models are evaluated on the GPU by libmev")

    def calculateSNR(self, bs, ue):
        raise NotImplementedError("channel models are evaluated on the GPU by libmev")

    @classmethod
    def datarate(cls, bs, ue, snr):
        raise NotImplementedError("channel models are evaluated on the GPU by libmev")

    def lower_params(self) -> dict:
        raise NotImplementedError(
            f"{type(self).__name__}: only OkumuraHata has a device lowering")


class OkumuraHata(Channel):
    def lower_params(self) -> dict:
        return {"channel": "okumura_hata"}
