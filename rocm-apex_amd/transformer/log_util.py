"""Transformer logging helpers (reference apex/transformer/log_util.py)."""
import logging
import os


def get_transformer_logger(name: str) -> logging.Logger:
    name_wo_ext = os.path.splitext(name)[0]
    return logging.getLogger(name_wo_ext)


def set_logging_level(verbosity) -> None:
    """Change the severity of the library root logger (``apex``)."""
    logging.getLogger("apex").setLevel(verbosity)
