"""scripts/ab_frame_cook.py with the fused framing cook off (RSMI_FENC_FUSE=0):
the unfused side of the A/B (k_frame, encode, one cook over every packet)."""
import os
import runpy

os.environ["RSMI_FENC_FUSE"] = "0"
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "ab_frame_cook.py"), run_name="__main__")
