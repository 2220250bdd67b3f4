"""Fully-connected model family (the only model family of the reference).

The reference describes a network purely through its JSON config: a list of layers, each with
``nodes`` output units, per-neuron ``weights``/``bias`` and an ``activation``
(/root/reference/config/config_sample.json:1-33); hidden layers use ReLU and the output layer
softmax (/root/reference/scripts/generate_mnist_pytorch.py:22-33, notebook export
``…ipynb:464-506``). :class:`MLPSpec` is that description without the weights; it also parses
the compact ``784-512-256-128-10`` form used by BASELINE.json and names the benchmark configs.
"""
from __future__ import annotations

import re
from dataclasses import dataclass, field
from typing import Iterable, Sequence

# Activation names as written in the reference JSON (case-sensitive in the stage worker,
# /root/reference/src/grpc_node.py:62-73; anything unknown behaves as identity).
ACTIVATIONS = ("linear", "relu", "sigmoid", "softmax")
ACT_CODE = {"linear": 0, "relu": 1, "sigmoid": 2, "softmax": 3}


def normalize_activation(name: str | None, case_sensitive: bool = True) -> str:
    """Map a JSON activation string onto the engine's activation set.

    The stage worker compares names case-sensitively and treats anything else as linear
    (grpc_node.py:64-73); ``manual_nn.py`` lowercases first (scripts/manual_nn.py:66).
    """
    if name is None:
        return "linear"
    key = name if case_sensitive else name.lower()
    return key if key in ACTIVATIONS else "linear"


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass(frozen=True)
class LayerSpec:
    in_dim: int
    out_dim: int
    activation: str = "relu"
    type: str = "hidden"

    def __post_init__(self):
        if self.in_dim <= 0 or self.out_dim <= 0:
            raise ValueError(f"layer dims must be positive, got {self.in_dim}->{self.out_dim}")
        if self.activation not in ACTIVATIONS:
            raise ValueError(f"unknown activation {self.activation!r}")

    @property
    def params(self) -> int:
        return self.in_dim * self.out_dim + self.out_dim

    @property
    def flops_per_sample_train(self) -> int:
        """fwd + dgrad + wgrad multiply-adds x2 (dgrad counted even for a first layer)."""
        return 6 * self.in_dim * self.out_dim


@dataclass(frozen=True)
class MLPSpec:
    layers: tuple[LayerSpec, ...]
    name: str = ""

    def __post_init__(self):
        if not self.layers:
            raise ValueError("an MLP needs at least one layer")
        for a, b in zip(self.layers, self.layers[1:]):
            if a.out_dim != b.in_dim:
                raise ValueError(f"layer width mismatch: {a.out_dim} feeds {b.in_dim}")

    @property
    def in_dim(self) -> int:
        return self.layers[0].in_dim

    @property
    def out_dim(self) -> int:
        return self.layers[-1].out_dim

    @property
    def widths(self) -> list[int]:
        return [self.layers[0].in_dim] + [l.out_dim for l in self.layers]

    @property
    def num_params(self) -> int:
        return sum(l.params for l in self.layers)

    def flops_per_sample_train(self) -> int:
        """EXECUTED training FLOPs per sample: fwd + dgrad + wgrad of every layer, minus the
        first layer's dgrad (the gradient w.r.t. the input data is never computed)."""
        first = self.layers[0]
        return sum(l.flops_per_sample_train for l in self.layers) - \
            2 * first.in_dim * first.out_dim

    def describe(self) -> str:
        return "-".join(str(w) for w in self.widths)

    @staticmethod
    def from_widths(widths: Sequence[int], hidden_act: str = "relu", out_act: str = "softmax",
                    name: str = "") -> "MLPSpec":
        if len(widths) < 2:
            raise ValueError("need at least input and output widths")
        layers = []
        for i in range(len(widths) - 1):
            last = i == len(widths) - 2
            layers.append(LayerSpec(int(widths[i]), int(widths[i + 1]),
                                    out_act if last else hidden_act,
                                    "output" if last else "hidden"))
        return MLPSpec(tuple(layers), name or "-".join(map(str, widths)))

    @staticmethod
    def parse(text: str) -> "MLPSpec":
        """``"784-512-256-128-10"``; repetition ``"784-1024x7-10"`` (or ×) expands a width."""
        if text in NAMED_MODELS:
            return NAMED_MODELS[text]
        widths: list[int] = []
        for tok in re.split(r"-", text.strip()):
            m = re.fullmatch(r"(\d+)\s*(?:[x×\*]\s*(\d+))?", tok.strip())
            if not m:
                raise ValueError(f"cannot parse model spec {text!r} (token {tok!r})")
            widths += [int(m.group(1))] * (int(m.group(2)) if m.group(2) else 1)
        return MLPSpec.from_widths(widths, name=text)


# BASELINE.json configs ("784-1024x6-10" has 7 Linear layers; the 8-stage
# one-layer-per-GPU pipeline uses 784-1024x7-10 = 8 Linear layers).
NAMED_MODELS: dict[str, MLPSpec] = {}


def _register(name: str, widths: Iterable[int]) -> None:
    NAMED_MODELS[name] = MLPSpec.from_widths(list(widths), name=name)


_register("mnist-784-128-10", [784, 128, 10])                 # config 1 (manual_nn CPU path)
_register("mnist-fcnn", [784, 512, 256, 128, 10])             # config 2 (4-stage)
_register("mlp8", [784] + [1024] * 7 + [10])                  # config 3 (8-stage, 8 Linear)
_register("mlp7", [784] + [1024] * 6 + [10])                  # config 3 literal (7 Linear)
_register("wide", [784, 8192, 8192, 10])                      # config 4 (PP=2 x DP=4)
_register("notebook", [784, 32, 16, 10])                      # notebook recipe (…ipynb:274-285)
_register("pytorch-recipe", [784, 128, 64, 10])               # generate_mnist_pytorch.py:22-33


@dataclass
class LayerGeom:
    """Padded device geometry of one layer (MFMA tiles need multiples of 64)."""

    index: int  # global layer index
    spec: LayerSpec
    kp: int = field(init=False)
    np_: int = field(init=False)

    def __post_init__(self):
        self.kp = round_up(self.spec.in_dim, 64)
        self.np_ = round_up(self.spec.out_dim, 64)
