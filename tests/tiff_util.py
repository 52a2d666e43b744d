"""The tests' TIFF writer: floodgan.data.write_tile (tifffile.imsave's layout for dataset tiles); the
decoder is also checked against PIL, an independent writer (tests/test_data_cpu.py)."""
from floodgan.data import write_tile as write_tiff  # noqa: F401
