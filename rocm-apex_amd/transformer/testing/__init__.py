"""Standalone Megatron models, arguments and globals for the transformer tests
(reference apex/transformer/testing/)."""
