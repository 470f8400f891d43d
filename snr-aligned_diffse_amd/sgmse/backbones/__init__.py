from .shared import BackboneRegistry
from .ncsnpp import NCSNpp
from .snrnet import SNRNet

__all__ = ["BackboneRegistry", "NCSNpp", "SNRNet"]
