"""Mirror of the reference's ``cost_volume`` package (the four standalone CV modules)."""
from .concatenate import TorchConcatenateCost
from .groupwise import TorchGroupwiseCost
from .inner_product import TorchInnerProductCost
from .interweave import TorchInterweaveCost

__all__ = ["TorchConcatenateCost", "TorchGroupwiseCost", "TorchInnerProductCost", "TorchInterweaveCost"]
