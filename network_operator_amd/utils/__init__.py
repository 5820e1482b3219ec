from .paths import BIN_DIR, LIB_DIR, PACKAGE_DIR, REPO_ROOT, NativeArtifactMissing, hip_library, native_bin

__all__ = ["BIN_DIR", "LIB_DIR", "PACKAGE_DIR", "REPO_ROOT", "NativeArtifactMissing", "hip_library", "native_bin"]
