"""expertsim — MI355X-native (gfx950 HIP) implementation of the expertsim MoE-GAN training step.

Drop-in for the reference's Python API (patrick-bedkowski/Generative-DNN-for-Physics-Simulations-
CERN): ``expertsim.models`` (registry + model classes), ``expertsim.models.moe.MoEWrapper``,
``expertsim.train`` (loop / optimizers) and ``expertsim/config/default.yaml``.  All arithmetic of
the training step runs in the HIP kernels of ``csrc/`` through the C ABI in
``include/expertsim_hip.h``; see DESIGN.md.
"""
__version__ = "0.1.0"
