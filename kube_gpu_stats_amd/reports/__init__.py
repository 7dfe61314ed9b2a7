"""The reference's two reports, rebuilt: ``who_use_gpu`` (F1) and ``gpu_util_stats`` (F2-F4)."""
