from .batch_norm import BatchNorm2d_NHWC, bn_add_bn_relu, bn_nhwc_function, bn_relu_maxpool  # noqa: F401
