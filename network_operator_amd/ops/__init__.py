"""HIP/gfx950 kernels used to validate the scale-out fabric the operator configures."""

from .hip import HipError, copy, fill_expected_sum, fill_pattern, verify_sum, xgmi_probe

__all__ = ["HipError", "copy", "fill_expected_sum", "fill_pattern", "verify_sum", "xgmi_probe"]
