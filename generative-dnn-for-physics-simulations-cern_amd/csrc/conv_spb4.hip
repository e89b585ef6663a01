// The 4-wave split-fp32 FWD / DGRAD kernels (conv_ring_kernel SPL = 3) in a translation unit of their
// own, built with VGPR-form MFMA and without SLP vectorisation (Makefile; reasons at es_spb4_launch).
#define ES_SPB4_TU 1
#include "conv_mfma.hip"
