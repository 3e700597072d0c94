"""Scene JSON -> HDF5 CLI, flag-compatible with the reference `scene_processor/convert_scene.py:11-45`.

    python convert_scene.py examples/cbox.json [--output_h5_path cbox.h5] [--mesh_path IGNORED.obj]

Restated without trimesh/h5py/dacite in renderformer_amd.scene_convert (smooth-shading normals: parity
unpinned, see that module).  --mesh_path is accepted for compatibility; no intermediate meshes are written.
"""
from __future__ import annotations

import argparse
import sys

from renderformer_amd.scene_convert import convert_scene


def main(argv=None):
    parser = argparse.ArgumentParser(description="Convert scene config to mesh and h5")
    parser.add_argument("scene_config_path", type=str, help="Path to scene config JSON file")
    parser.add_argument("--mesh_path", type=str, default=None,
                        help="accepted for compatibility (no intermediate mesh file is written)")
    parser.add_argument("--output_h5_path", type=str, default=None,
                        help="Output path for h5 file. If not provided, will use scene_config_path with .h5 extension")
    args = parser.parse_args(argv)
    out = convert_scene(args.scene_config_path, args.output_h5_path)
    print(f"Done converting scene config to h5 file: {out}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
