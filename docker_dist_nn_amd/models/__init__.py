from .mlp import (ACT_CODE, ACTIVATIONS, NAMED_MODELS, LayerGeom, LayerSpec, MLPSpec,
                  normalize_activation, round_up)

__all__ = ["ACT_CODE", "ACTIVATIONS", "NAMED_MODELS", "LayerGeom", "LayerSpec", "MLPSpec",
           "normalize_activation", "round_up"]
