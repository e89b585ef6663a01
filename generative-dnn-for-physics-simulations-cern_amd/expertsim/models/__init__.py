"""Model registry — reference: expertsim/models/__init__.py:11-28.

Same keys and ``build_model(name, specs, device)`` contract.  The reference's registry also lists
``proton.generator_unified`` and ``router_attention`` whose classes do not exist (its package import
fails with AttributeError, models/__init__.py:13,21) and the unused ``DiscriminatorUnified``; those
three entries are not part of the training step and are omitted.

``neutron56.*`` is the build's declared 56x56 shape extension for BASELINE configs[4] (SURVEY.md
§8(d) C5: no reference model accepts 56x56) -- throughput-only, parity unpinned."""
import torch

from .neutron.aux_reg import AuxRegNeutron
from .neutron.discriminator import DiscriminatorNeutron, DiscriminatorNeutron56
from .neutron.generator import GeneratorNeutron, GeneratorNeutron56
from .proton.aux_reg import AuxReg
from .proton.discriminator import Discriminator
from .proton.generator import Generator
from .routers.router import RouterNetwork

MODEL_REGISTRY = {
    "proton.generator": Generator,
    "proton.discriminator": Discriminator,
    "proton.aux_reg": AuxReg,
    "neutron.generator": GeneratorNeutron,
    "neutron.discriminator": DiscriminatorNeutron,
    "neutron.aux_reg": AuxRegNeutron,
    "router_v1": RouterNetwork,
    "neutron56.generator": GeneratorNeutron56,
    "neutron56.discriminator": DiscriminatorNeutron56,
    "neutron56.aux_reg": AuxRegNeutron,
}


def build_model(name: str, model_specs: dict, device: torch.device):
    if name not in MODEL_REGISTRY:
        raise ValueError(f"Unknown model '{name}'. Available: {list(MODEL_REGISTRY.keys())}")
    return MODEL_REGISTRY[name](**model_specs).to(device)
