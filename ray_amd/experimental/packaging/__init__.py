from ray_amd.experimental.packaging.load_package import load_package  # noqa: F401
