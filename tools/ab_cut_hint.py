"""Run bench.py's config D / E legs with raster.CUT_SORT_HINT set (LDS sort class of the
depth-cut heads). usage: python tools/ab_cut_hint.py HINT [bench args...]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from my_depthsplat_amd import raster  # noqa: E402

raster.CUT_SORT_HINT = int(sys.argv[1])
sys.argv = [str(Path(__file__).resolve().parents[1] / "bench.py"), *sys.argv[2:]]
import bench  # noqa: E402

bench.main()
