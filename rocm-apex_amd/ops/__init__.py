"""Op layer: python entry points over the native gfx950 kernels plus torch reference paths."""
