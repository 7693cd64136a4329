"""torchmd-net_amd: MI355X-native hot path of TorchMD-NET (ET / TensorNet energy + forces).

Import name ``torchmdnet`` is kept so that code written against the reference
(``from torchmdnet.models.model import create_model``) runs unchanged; put the directory
``torchmd-net_amd`` on ``sys.path`` / ``PYTHONPATH``.
"""
__version__ = "0.1.0"
