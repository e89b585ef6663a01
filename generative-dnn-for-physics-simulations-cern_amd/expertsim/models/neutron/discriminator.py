"""Neutron-ZDC discriminator — reference: expertsim/models/neutron/discriminator.py:6-48.

44x44 input: SNconv3 -> 42x42 -> pool 2 -> 21x21 -> SNconv3 -> 19x19 -> pool 2 -> 9x9, flatten
16*9*9 = 1296 (the reference hard-codes flat_dim = 9*12*12 = 1296, discriminator.py:24).
"""
from ..sn_discriminator import SNDiscriminator


class DiscriminatorNeutron(SNDiscriminator):
    def __init__(self, cond_dim, **kwargs):
        super().__init__(cond_dim, image_shape=(44, 44), pool2=(2, 2))
        self.name = "Discriminator-neutron-1-expert-hinge-SN"


class DiscriminatorNeutron56(SNDiscriminator):
    """Declared 56x56 extension (BASELINE configs[4]): 56 -> 54 -> 27 -> 25 -> 12,
    flatten 16*12*12 = 2304.  No reference model: parity unpinned."""

    def __init__(self, cond_dim, **kwargs):
        super().__init__(cond_dim, image_shape=(56, 56), pool2=(2, 2))
        self.name = "Discriminator-neutron56-declared-extension"
