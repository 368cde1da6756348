"""MI355X-native data orchestration layer with Alluxio-compatible APIs."""
__version__ = "0.1.0"
