"""MI355X-native drop-in for the reference package ``ldpc_neural_decoder``.

Same module layout and public names as the reference's hot path (models.traditional_decoders,
models.message_gnn_decoder, utils.channel, utils.ldpc_utils); the compute runs in
libldpc_amd.so (HIP, gfx950) through the C ABI in include/ldpc_amd.h.
"""
__version__ = "0.1.0"
