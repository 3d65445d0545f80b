"""Drop-in for the ``Old/process_cloud.py`` CLI (--input --output --calib).

    python -m structured_light_for_3d_model_replication_amd.process_cloud --input scan/ --output out.ply

Same flags, defaults and behaviour (Old/process_cloud.py:221-236): errors are
printed, not raised.  Uses the fixed-threshold mask of that file (:47-49).
"""
from __future__ import annotations

import argparse

from .multi_point_cloud_process import gray_decode, load_calibration, reconstruct_point_cloud, save_ply


def main(argv=None):
    parser = argparse.ArgumentParser(description="Decode and Reconstruct 3D Scan")
    parser.add_argument("--input", required=True, help="Folder containing scan images")
    parser.add_argument("--output", default="output.ply", help="Output .ply file")
    parser.add_argument("--calib", default="./calib/calib_results/calib_cam_proj.mat",
                        help="Path to calibration mat file")
    args = parser.parse_args(argv)
    try:
        calib_data = load_calibration(args.calib)
        c_map, r_map, mask, texture = gray_decode(args.input)
        points, colors = reconstruct_point_cloud(c_map, r_map, mask, texture, calib_data)
        save_ply(points, colors, args.output)
        print("Done!")
    except Exception as e:  # noqa: BLE001 -- the reference prints every error (:235-236)
        print(f"Error: {e}")


if __name__ == "__main__":
    main()
