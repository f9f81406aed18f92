"""Benchmark model families: ResNet (ImageNet headline), and the transformer test models live in
apex.transformer.testing (GPT / BERT)."""
from .resnet import ResNet, resnet18, resnet34, resnet50, resnet101, resnet152  # noqa: F401
