"""ray_amd — an MI355X-native distributed ML runtime with Ray's API surface."""

__version__ = "0.1.0"
