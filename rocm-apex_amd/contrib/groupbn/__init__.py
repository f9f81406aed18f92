from .batch_norm import BatchNorm2d_NHWC, bn_nhwc_function  # noqa: F401
