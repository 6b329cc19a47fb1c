"""Wire / disk formats, host side (no device needed):
the binary PCD writer against the layout pcl::io::savePCDFileBinary produces
(header lines as post_process/merge_pcds.py:107-119 writes them, packed float32
records), and the reader's header pass."""
import numpy as np

from lio_gpu import formats as FM


def test_pcd_write_binary_layout(tmp_path):
    rng = np.random.default_rng(1)
    rec = rng.normal(0, 10, (1234, 4)).astype(np.float32)
    p = str(tmp_path / "m.pcd")
    FM.write_pcd_binary(p, rec)
    raw = open(p, "rb").read()
    header = (b"# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z intensity\n"
              b"SIZE 4 4 4 4\nTYPE F F F F\nCOUNT 1 1 1 1\nWIDTH 1234\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\n"
              b"POINTS 1234\nDATA binary\n")
    assert raw[: len(header)] == header
    assert raw[len(header):] == rec.tobytes()
    assert FM.pcd_points(p) == 1234


def test_pcd_reader_header_counts(tmp_path):
    p = str(tmp_path / "a.pcd")
    with open(p, "w") as f:
        f.write("# .PCD v0.7\nVERSION 0.7\nFIELDS x y z\nSIZE 4 4 4\nTYPE F F F\nCOUNT 1 1 1\nWIDTH 3\n"
                "HEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS 3\nDATA ascii\n1 2 3\n4 5 6\n7 8 9\n")
    assert FM.pcd_points(p) == 3
