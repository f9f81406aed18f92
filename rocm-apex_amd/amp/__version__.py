"""amp version (reference apex/amp/__version__.py)."""
VERSION = (0, 1, 0)
__version__ = ".".join(map(str, VERSION))
