"""Proton-ZDC discriminator — reference: expertsim/models/proton/discriminator.py:116-155.

56x30 input: SNconv3 -> 54x28 -> pool 2 -> 27x14 -> SNconv3 -> 25x12 -> pool (2,1) -> 12x12,
flatten 16*12*12 = 2304 (discriminator.py:134).
"""
from ..sn_discriminator import SNDiscriminator


class Discriminator(SNDiscriminator):
    def __init__(self, cond_dim, **kwargs):
        super().__init__(cond_dim, image_shape=(56, 30), pool2=(2, 1))
        self.name = "Discriminator-5-hinge-spectralnorm"
