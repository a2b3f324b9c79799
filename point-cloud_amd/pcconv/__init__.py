"""pcconv — Python host mirror of the reference `point-converter` library API
(point-converter/src/lib.rs, converter.rs) over the MI355X C ABI
(include/pcconv.h, libpcconv.so).

There is no CPU fallback: every call goes through the HIP build, and importing
this module fails loudly if libpcconv.so has not been built
(`make -C point-cloud_amd`, or `python -c "import __graft_entry__ as g; g.build()"`).

Reference-to-mirror map:
  convert_from_paths(paths, output)   lib.rs:11-60
  Converter(out_dir, ...)             lib.rs:86-101 load_metadata + converter.rs:79-94
  Converter.add_points(points)        converter.rs:106-112 (one call == one input file,
                                      ceil(n / batch_size) batches, lib.rs:31-52)
  Converter.finish()                  converter.rs:241-246 Drop (cells, then metadata.json)
  Converter(existing_dir)             incremental merge: lib.rs:86-101 + converter.rs:187-207
                                      (the directory's cells are the starting state)
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PCC_LIB") or os.path.join(HERE, "..", "build", "libpcconv.so")

POINT_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4"), ("rgba", "u1", (4,))])  # point.rs:8-14

# every symbol include/pcconv.h declares
EXPORTS = ["pcc_abi_version", "pcc_last_error", "pcc_options_default", "pcc_open", "pcc_add_points",
           "pcc_add_points_device", "pcc_add_empty_batches", "pcc_add_synthetic", "pcc_build", "pcc_write",
           "pcc_finish", "pcc_close", "pcc_get_stats", "pcc_set_profiling", "pcc_get_profile", "pcc_device_input",
           "pcc_convert_files", "pcc_shard_grid_from_bbox", "pcc_synth_device", "pcc_shard_bbox",
           "pcc_shard_bbox_nonfinite", "pcc_set_event_table", "pcc_shard_batch_starts",
           "pcc_shard_histogram", "pcc_shard_route", "pcc_declare_files", "pcc_add_keyed_points_device",
           "pcc_set_keyed_points_device", "pcc_input_landed", "pcc_set_level_range", "pcc_set_root_spill_batches",
           "pcc_pending_cells", "pcc_export_pending", "pcc_shard_slab_histogram", "pcc_shard_route_slabs", "pcc_shard_bbox_histogram", "pcc_shard_bbox_sample",
           "pcc_write_cell_view", "pcc_begin_file", "pcc_append_points", "pcc_end_file", "pcc_cancel_file",
           "pcc_set_summary", "pcc_write_cells", "pcc_write_metadata", "pcc_clear_input", "pcc_adopt_prior",
           "pcc_open_subtrees", "pcc_visit_cells", "pcc_shard_route_bitmaps", "pcc_shard_route_bitmaps_hist",
           "pcc_shard_keys_from_bitmaps",
           "pcc_release_device_cache", "pcc_grid_cells", "pcc_export_grid", "pcc_shard_resolve_buckets", "pcc_shard_lpt",
           "pcc_shard_plan_search"]


class Options(C.Structure):
    _fields_ = [("batch_size", C.c_uint32), ("device", C.c_int32), ("cell_point_overflow_limit", C.c_uint32),
                ("sub_grid_dimension", C.c_uint32), ("max_cell_size", C.c_float), ("reserved", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("number_of_points", C.c_uint64), ("hierarchies", C.c_uint32), ("levels", C.c_uint32),
                ("cells", C.c_uint64), ("slabs", C.c_uint64), ("arrivals", C.c_uint64),
                ("grid_points", C.c_uint64), ("kept_points", C.c_uint64), ("build_ms", C.c_double),
                ("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3), ("level0_early_tiles", C.c_uint64),
                ("level0_fold", C.c_uint32), ("sequential_replay", C.c_uint32)]

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_ if not k.startswith("bbox")}
        d["bbox_min"] = list(self.bbox_min)
        d["bbox_max"] = list(self.bbox_max)
        return d


class Profile(C.Structure):
    _fields_ = [("level0_ms", C.c_double), ("dense_ms", C.c_double), ("small_ms", C.c_double),
                ("bucket_ms", C.c_double), ("next_ms", C.c_double), ("dense_arrivals", C.c_uint64),
                ("small_arrivals", C.c_uint64), ("dense_launches", C.c_uint32), ("small_launches", C.c_uint32)]


class ShardGrid(C.Structure):
    """pcc_shard_grid: level-0 cell grid spanned by the global bounding box."""
    _fields_ = [("lo", C.c_int32 * 3), ("dims", C.c_uint32 * 3), ("cell_size", C.c_float)]

    @property
    def ncells(self) -> int:
        return int(self.dims[0]) * int(self.dims[1]) * int(self.dims[2])


class CellView(C.Structure):
    """pcc_cell_view: one built cell in memory (cell.rs:33-38, Header cell.rs:238-261)."""
    _fields_ = [("hierarchy", C.c_uint32), ("x", C.c_int32), ("y", C.c_int32), ("z", C.c_int32),
                ("total_number_of_points", C.c_uint32), ("number_of_points", C.c_uint32),
                ("number_of_overflow_points", C.c_uint32), ("size", C.c_float), ("sub_cell_size", C.c_float),
                ("pos", C.c_float * 3), ("grid", C.c_void_p), ("entries", C.c_uint32),
                ("child", (C.c_int32 * 3) * 8), ("count", C.c_uint32 * 8), ("list", C.c_void_p * 8)]

    def grid_points(self) -> np.ndarray:
        """Copy of the grid points (numpy POINT_DTYPE)."""
        n = int(self.number_of_points)
        if n == 0:
            return np.empty(0, dtype=POINT_DTYPE)
        return np.frombuffer((C.c_char * (16 * n)).from_address(self.grid), dtype=POINT_DTYPE).copy()

    def overflow(self) -> list:
        """[(child index, None | numpy list in stored order)] (cell.rs:108-153 entries)."""
        out = []
        for e in range(int(self.entries)):
            n = int(self.count[e])
            lst = None if n == 0 else np.frombuffer((C.c_char * (16 * n)).from_address(self.list[e]),
                                                    dtype=POINT_DTYPE).copy()
            out.append((tuple(self.child[e]), lst))
        return out


CELL_VISITOR = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p)


class PccError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"pcconv error {code}: {msg}")
        self.code = code


_lib = None


def lib():
    """Load libpcconv.so (no fallback: raises if the HIP library is missing)."""
    global _lib
    if _lib is None:
        path = os.path.abspath(LIB_PATH)
        if not os.path.exists(path):
            raise ImportError(f"libpcconv.so not built at {path}; run `make -C point-cloud_amd`")
        L = C.CDLL(path)
        vp = C.c_void_p
        L.pcc_abi_version.restype = C.c_uint32
        L.pcc_last_error.restype = C.c_char_p
        L.pcc_options_default.argtypes = [C.POINTER(Options)]
        L.pcc_open.argtypes = [C.c_char_p, C.POINTER(Options), C.POINTER(vp)]
        L.pcc_open_subtrees.argtypes = [C.c_char_p, C.POINTER(Options), vp, C.c_uint64, C.POINTER(vp)]
        L.pcc_add_points.argtypes = [vp, vp, C.c_uint64]
        L.pcc_add_points_device.argtypes = [vp, vp, C.c_uint64]
        L.pcc_add_empty_batches.argtypes = [vp, C.c_uint32]
        L.pcc_add_synthetic.argtypes = [vp, C.c_uint64, C.c_int, C.c_uint64, C.c_float, C.c_float]
        L.pcc_build.argtypes = [vp]
        L.pcc_write.argtypes = [vp]
        L.pcc_finish.argtypes = [vp]
        L.pcc_close.argtypes = [vp]
        L.pcc_get_stats.argtypes = [vp, C.POINTER(Stats)]
        L.pcc_set_profiling.argtypes = [vp, C.c_int]
        L.pcc_get_profile.argtypes = [vp, C.POINTER(Profile)]
        L.pcc_device_input.argtypes = [vp]
        L.pcc_device_input.restype = vp
        L.pcc_convert_files.argtypes = [C.c_char_p, C.POINTER(C.c_char_p), C.c_size_t, C.POINTER(Options)]
        f3 = C.POINTER(C.c_float)
        L.pcc_shard_grid_from_bbox.argtypes = [f3, f3, C.c_float, C.POINTER(ShardGrid)]
        L.pcc_synth_device.argtypes = [vp, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.c_float, C.c_float, C.c_int]
        L.pcc_shard_bbox.argtypes = [vp, C.c_uint64, f3, f3, C.c_int]
        L.pcc_shard_bbox_nonfinite.argtypes = [vp, C.c_uint64, f3, C.c_int]
        L.pcc_set_event_table.argtypes = [vp, vp, vp, C.c_uint64, C.c_uint64]
        L.pcc_shard_batch_starts.argtypes = [vp, vp, vp, C.c_uint32, vp, C.c_uint64, vp, C.c_int]
        L.pcc_shard_histogram.argtypes = [vp, C.c_uint64, C.POINTER(ShardGrid), vp, C.c_int]
        L.pcc_shard_route.argtypes = [vp, C.c_uint64, C.c_uint32, C.POINTER(ShardGrid), vp, C.c_uint32, vp, vp,
                                      C.POINTER(C.c_uint64), C.c_int]
        L.pcc_declare_files.argtypes = [vp, C.POINTER(C.c_uint64), C.c_uint64]
        L.pcc_add_keyed_points_device.argtypes = [vp, vp, vp, C.c_uint64]
        L.pcc_set_keyed_points_device.argtypes = [vp, vp, vp, C.c_uint64]
        L.pcc_input_landed.argtypes = [vp, C.c_uint64, C.c_uint64, vp]
        L.pcc_set_level_range.argtypes = [vp, C.c_uint32, C.c_uint32, C.c_int]
        L.pcc_shard_slab_histogram.argtypes = [vp, C.c_uint64, C.POINTER(ShardGrid), C.c_uint32, vp, C.c_int]
        L.pcc_shard_bbox_histogram.argtypes = [vp, C.c_uint64, C.POINTER(ShardGrid), C.c_uint32, vp, f3, f3,
                                               C.POINTER(C.c_uint64), C.c_int]
        L.pcc_shard_bbox_sample.argtypes = [vp, C.c_uint64, f3, f3, C.c_int]
        L.pcc_shard_route_slabs.argtypes = [vp, C.c_uint64, C.c_uint32, C.POINTER(ShardGrid), C.c_uint32, vp,
                                            C.c_uint32, vp, vp, C.POINTER(C.c_uint64), C.c_int]
        L.pcc_shard_route_bitmaps.argtypes = [vp, C.c_uint64, C.POINTER(ShardGrid), C.c_uint32, vp, C.c_uint32, vp,
                                              vp, C.POINTER(C.c_uint64), C.c_int]
        L.pcc_shard_route_bitmaps_hist.argtypes = [vp, C.c_uint64, C.POINTER(ShardGrid), C.c_uint32, vp, C.c_uint32,
                                                   vp, vp, vp, C.POINTER(C.c_uint64), C.c_int]
        L.pcc_shard_keys_from_bitmaps.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint32, vp,
                                                  C.c_uint64, C.c_int]
        L.pcc_write_cell_view.argtypes = [C.c_char_p, vp]
        L.pcc_begin_file.argtypes = [vp, C.c_uint64]
        L.pcc_append_points.argtypes = [vp, vp, C.c_uint64]
        L.pcc_end_file.argtypes = [vp, C.c_uint64]
        L.pcc_cancel_file.argtypes = [vp]
        L.pcc_set_root_spill_batches.argtypes = [vp, vp, vp, C.c_uint64]
        L.pcc_pending_cells.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.pcc_export_pending.argtypes = [vp, vp, vp, vp, vp, vp]
        L.pcc_shard_lpt.argtypes = [vp, C.c_uint64, C.c_uint32, vp, vp]
        L.pcc_shard_plan_search.argtypes = [vp, vp, vp, vp, vp, C.c_uint32, C.c_uint32, C.c_uint32,
                                            C.POINTER(C.c_uint32), C.POINTER(C.c_double), vp, vp, vp, vp, vp]
        L.pcc_grid_cells.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.pcc_export_grid.argtypes = [vp, vp, vp, vp]
        L.pcc_shard_resolve_buckets.argtypes = [vp, vp, C.c_uint64, C.c_uint32, vp, vp, vp, C.c_uint64, C.c_uint32,
                                                C.c_uint32, vp, vp, vp, vp, vp, vp, C.POINTER(C.c_uint64),
                                                C.POINTER(C.c_uint64), C.c_int]
        L.pcc_set_summary.argtypes = [vp, C.c_uint64, f3, f3, C.c_uint32]
        L.pcc_write_cells.argtypes = [vp]
        L.pcc_write_metadata.argtypes = [vp]
        L.pcc_clear_input.argtypes = [vp]
        L.pcc_adopt_prior.argtypes = [vp, vp]
        L.pcc_visit_cells.argtypes = [vp, CELL_VISITOR, vp]
        L.pcc_release_device_cache.argtypes = []
        L.pcc_release_device_cache.restype = C.c_uint64
        _lib = L
    return _lib


def _check(rc: int):
    if rc != 0:
        raise PccError(rc, lib().pcc_last_error().decode(errors="replace"))


def release_device_cache() -> int:
    """Frees the device buffers closed converters left cached; returns the bytes freed."""
    return int(lib().pcc_release_device_cache())


def default_options(**kw) -> Options:
    o = Options()
    _check(lib().pcc_options_default(C.byref(o)))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


class Converter:
    """converter.rs:72-94 Converter, built on the GPU at finish()/build()."""

    def __init__(self, out_dir: str, batch_size: int = 10_000, device: int = 0, config: dict | None = None,
                 subtrees=None):
        """`subtrees` (sharded merge, pcc_open_subtrees): level-0 cell triples
        whose existing cells this converter loads and rewrites."""
        opt = default_options(batch_size=batch_size, device=device, **(config or {}))
        h = C.c_void_p()
        if subtrees is None:
            _check(lib().pcc_open(os.fsencode(out_dir), C.byref(opt), C.byref(h)))
        else:
            st = np.ascontiguousarray(np.asarray(subtrees, dtype=np.int32).reshape(-1, 3))
            _check(lib().pcc_open_subtrees(os.fsencode(out_dir), C.byref(opt), st.ctypes.data, len(st), C.byref(h)))
        self._h = h
        self.out_dir = out_dir

    def add_points(self, pts: np.ndarray):
        """One input file (host array of POINT_DTYPE)."""
        pts = np.ascontiguousarray(pts, dtype=POINT_DTYPE)
        _check(lib().pcc_add_points(self._h, pts.ctypes.data, len(pts)))

    def add_file_pieces(self, pieces, keep: int | None = None):
        """One file delivered in pieces (pcc_begin_file / pcc_append_points /
        pcc_end_file): the concatenation of `pieces` (numpy POINT arrays), or its
        first `keep` points."""
        import numpy as _np
        pieces = [_np.ascontiguousarray(p) for p in pieces]
        total = sum(len(p) for p in pieces)
        _check(lib().pcc_begin_file(self._h, total))
        for p in pieces:
            _check(lib().pcc_append_points(self._h, C.c_void_p(p.ctypes.data), len(p)))
        _check(lib().pcc_end_file(self._h, total if keep is None else keep))

    def add_points_device(self, dev_ptr: int, n: int):
        _check(lib().pcc_add_points_device(self._h, C.c_void_p(dev_ptr), n))

    def add_empty_batches(self, k: int):
        _check(lib().pcc_add_empty_batches(self._h, k))

    def add_synthetic(self, seed: int, kind: int, n: int, lo: float = -1000.0, extent: float = 2000.0):
        _check(lib().pcc_add_synthetic(self._h, seed, kind, n, lo, extent))

    def build(self) -> dict:
        _check(lib().pcc_build(self._h))
        return self.stats()

    def write(self):
        _check(lib().pcc_write(self._h))

    def stats(self) -> dict:
        s = Stats()
        _check(lib().pcc_get_stats(self._h, C.byref(s)))
        return s.as_dict()

    def set_profiling(self, on: bool = True):
        _check(lib().pcc_set_profiling(self._h, 1 if on else 0))

    def kernel_times(self) -> dict:
        p = Profile()
        _check(lib().pcc_get_profile(self._h, C.byref(p)))
        return {k: getattr(p, k) for k, _ in p._fields_}

    def device_input(self) -> int:
        return lib().pcc_device_input(self._h)

    # ---- sharded build (driven by pcconv.dist)
    def declare_files(self, file_points):
        arr = (C.c_uint64 * len(file_points))(*[int(v) for v in file_points])
        _check(lib().pcc_declare_files(self._h, arr, len(file_points)))

    def set_event_table(self, starts, batches, total_batches: int):
        """Rank-local keys: point i's event batch is batches[k] for the last k with
        starts[k] <= i (pcc_set_event_table); then set_keyed_points_device(ptr, 0, n)."""
        st = np.ascontiguousarray(starts, dtype=np.uint64)
        eb = np.ascontiguousarray(batches, dtype=np.uint32)
        _check(lib().pcc_set_event_table(self._h, st.ctypes.data, eb.ctypes.data, len(st), int(total_batches)))

    def add_keyed_points_device(self, pts_ptr: int, keys_ptr: int, n: int):
        _check(lib().pcc_add_keyed_points_device(self._h, C.c_void_p(pts_ptr), C.c_void_p(keys_ptr), n))

    def set_level_range(self, root_level: int, max_levels: int, raw: bool = False):
        _check(lib().pcc_set_level_range(self._h, root_level, max_levels, 1 if raw else 0))

    def set_root_spill_batches(self, cells_xyz, spill_batch):
        xyz = np.ascontiguousarray(cells_xyz, dtype=np.int32).reshape(-1, 3)
        sb = np.ascontiguousarray(spill_batch, dtype=np.uint32).reshape(-1)
        _check(lib().pcc_set_root_spill_batches(self._h, xyz.ctypes.data, sb.ctypes.data, len(sb)))

    def pending_cells(self) -> tuple[int, int]:
        nc, npt = C.c_uint64(0), C.c_uint64(0)
        _check(lib().pcc_pending_cells(self._h, C.byref(nc), C.byref(npt)))
        return nc.value, npt.value

    def export_pending(self, pts_ptr: int, keys_ptr: int):
        """(cells (n,3) int32, spill batches (n,) uint32, points per cell (n,)
        uint64); the arrivals go to the device buffers (pending_cells()[1] each)."""
        nc, _ = self.pending_cells()
        xyz = np.zeros((nc, 3), dtype=np.int32)
        sb = np.zeros(nc, dtype=np.uint32)
        cn = np.zeros(nc, dtype=np.uint64)
        _check(lib().pcc_export_pending(self._h, xyz.ctypes.data, sb.ctypes.data, cn.ctypes.data, C.c_void_p(pts_ptr),
                                        C.c_void_p(keys_ptr)))
        return xyz, sb, cn

    def grid_cells(self) -> tuple[int, int]:
        nc, npt = C.c_uint64(0), C.c_uint64(0)
        _check(lib().pcc_grid_cells(self._h, C.byref(nc), C.byref(npt)))
        return nc.value, npt.value

    def export_grid(self, pts_ptr: int):
        """pcc_export_grid: (cells (n,3) int32, grid points per cell (n,) uint64);
        the points go to the device buffer (grid_cells()[1] rows)."""
        nc, _ = self.grid_cells()
        xyz = np.zeros((nc, 3), dtype=np.int32)
        cn = np.zeros(nc, dtype=np.uint64)
        _check(lib().pcc_export_grid(self._h, xyz.ctypes.data, cn.ctypes.data, C.c_void_p(pts_ptr)))
        return xyz, cn

    def set_keyed_points_device(self, pts_ptr: int, keys_ptr: int, n: int):
        """Borrow (no copy) this rank's keyed input until build() returns."""
        _check(lib().pcc_set_keyed_points_device(self._h, C.c_void_p(pts_ptr), C.c_void_p(keys_ptr), n))

    def input_landed(self, first: int, last: int, after_stream: int = 0):
        """pcc_input_landed: points [first, last) of the borrowed input are in
        place once after_stream's queued work completes; level-0 pass 1 of
        their groups runs behind it (sharded exchange)."""
        _check(lib().pcc_input_landed(self._h, first, last, C.c_void_p(after_stream or None)))

    def set_summary(self, number_of_points: int, bmin, bmax, hierarchies: int):
        _check(lib().pcc_set_summary(self._h, number_of_points, (C.c_float * 3)(*bmin), (C.c_float * 3)(*bmax),
                                     hierarchies))

    def write_cells(self):
        _check(lib().pcc_write_cells(self._h))

    def write_metadata(self):
        _check(lib().pcc_write_metadata(self._h))

    def clear_input(self):
        _check(lib().pcc_clear_input(self._h))

    def adopt_prior(self, other: "Converter"):
        """Incremental merge without files: `other`'s built cloud becomes this
        (freshly opened) converter's existing cloud, as if it had been written to
        this converter's directory before opening it (lib.rs:86-101)."""
        _check(lib().pcc_adopt_prior(self._h, other._h))

    def visit_cells(self, fn):
        """Calls fn(view_ptr) for every built cell (pcc_visit_cells; the view is a
        CellView valid during the call only: `CellView.from_address(view_ptr)`).
        A nonzero return stops the walk and raises PccError with that code."""
        err = []

        def cb(view, _user):
            try:
                return int(fn(view) or 0)
            except BaseException as e:   # never unwind through the C frames
                err.append(e)
                return -1
        rc = lib().pcc_visit_cells(self._h, CELL_VISITOR(cb), None)
        if err:
            raise err[0]
        _check(rc)

    def finish(self):
        """converter.rs:241-246 Drop: build if needed, write cells then metadata.json."""
        h, self._h = self._h, None
        if h:
            _check(lib().pcc_finish(h))

    def close(self):
        h, self._h = self._h, None
        if h:
            lib().pcc_close(h)

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        if exc_type is None:
            self.finish()
        else:
            self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def shard_grid_from_bbox(gmin, gmax, max_cell_size: float = 1000.0) -> ShardGrid:
    g = ShardGrid()
    _check(lib().pcc_shard_grid_from_bbox((C.c_float * 3)(*gmin), (C.c_float * 3)(*gmax), max_cell_size, C.byref(g)))
    return g


def synth_device(dst_ptr: int, first: int, n: int, seed: int, kind: int = 0, lo: float = -1000.0,
                 extent: float = 2000.0, device: int = 0):
    _check(lib().pcc_synth_device(C.c_void_p(dst_ptr), first, n, seed, kind, lo, extent, device))


EDOM = 33   # pcc_shard_bbox*: the input has NaN or infinite coordinates


def _check_edom(rc: int) -> bool:
    """False when rc is -EDOM (NaN / infinite coordinates: shard_bbox_nonfinite)."""
    if rc == -EDOM:
        return False
    _check(rc)
    return True


def shard_bbox(pts_ptr: int, n: int, device: int = 0):
    """(bmin, bmax), or None when a coordinate is NaN or infinite."""
    bmin, bmax = (C.c_float * 3)(), (C.c_float * 3)()
    if not _check_edom(lib().pcc_shard_bbox(C.c_void_p(pts_ptr), n, bmin, bmax, device)):
        return None
    return list(bmin), list(bmax)


def shard_batch_starts(bm_ptr: int, nwords, key0, gstarts, device: int = 0) -> np.ndarray:
    """Rank-local start of every global batch start key (pcc_shard_batch_starts)."""
    nw = np.ascontiguousarray(nwords, dtype=np.uint64)
    k0 = np.ascontiguousarray(key0, dtype=np.uint64)
    gs = np.ascontiguousarray(gstarts, dtype=np.uint64)
    out = np.empty(len(gs), dtype=np.uint64)
    _check(lib().pcc_shard_batch_starts(C.c_void_p(bm_ptr), nw.ctypes.data, k0.ctypes.data, len(nw), gs.ctypes.data,
                                        len(gs), out.ctypes.data, device))
    return out


def shard_bbox_nonfinite(pts_ptr: int, n: int, device: int = 0) -> list:
    """The 15 values of pcc_shard_bbox_nonfinite: the reference's box over the
    non-NaN values, which axes have one, and the cell extent of the points with
    no infinite coordinate (NaN as 0)."""
    parts = (C.c_float * 15)()
    _check(lib().pcc_shard_bbox_nonfinite(C.c_void_p(pts_ptr), n, parts, device))
    return list(parts)


def shard_histogram(pts_ptr: int, n: int, grid: ShardGrid, hist_ptr: int, device: int = 0):
    _check(lib().pcc_shard_histogram(C.c_void_p(pts_ptr), n, C.byref(grid), C.c_void_p(hist_ptr), device))


SHARD_LAYERS = 256   # PCC_SHARD_LAYERS
SHARD_LDS_UNITS = 16384   # engine.hip kShLds: slab units a fused bbox+histogram pass counts in LDS


def shard_slab_histogram(pts_ptr: int, n: int, grid: ShardGrid, sub_grid_dimension: int, hist_ptr: int,
                         device: int = 0):
    _check(lib().pcc_shard_slab_histogram(C.c_void_p(pts_ptr), n, C.byref(grid), sub_grid_dimension,
                                          C.c_void_p(hist_ptr), device))


def shard_bbox_histogram(pts_ptr: int, n: int, grid: ShardGrid, sub_grid_dimension: int, hist_ptr: int,
                         device: int = 0):
    """(bmin, bmax, outside): local box + histogram over a guessed grid, one pass;
    None when a coordinate is NaN or infinite."""
    bmin, bmax, out = (C.c_float * 3)(), (C.c_float * 3)(), C.c_uint64(0)
    if not _check_edom(lib().pcc_shard_bbox_histogram(C.c_void_p(pts_ptr), n, C.byref(grid), sub_grid_dimension,
                                                      C.c_void_p(hist_ptr), bmin, bmax, C.byref(out), device)):
        return None
    return list(bmin), list(bmax), int(out.value)


def shard_bbox_sample(pts_ptr: int, n: int, device: int = 0):
    """(bmin, bmax) of the sample, or None when it is not finite."""
    bmin, bmax = (C.c_float * 3)(), (C.c_float * 3)()
    if not _check_edom(lib().pcc_shard_bbox_sample(C.c_void_p(pts_ptr), n, bmin, bmax, device)):
        return None
    return list(bmin), list(bmax)


def shard_route_slabs(pts_ptr: int, n: int, key0: int, grid: ShardGrid, sub_grid_dimension: int, owner_ptr: int,
                      nranks: int, send_ptr: int, keys_ptr: int, device: int = 0):
    counts = (C.c_uint64 * nranks)()
    _check(lib().pcc_shard_route_slabs(C.c_void_p(pts_ptr), n, key0, C.byref(grid), sub_grid_dimension,
                                       C.c_void_p(owner_ptr), nranks, C.c_void_p(send_ptr), C.c_void_p(keys_ptr),
                                       counts, device))
    return [int(c) for c in counts]


def shard_route_bitmaps(pts_ptr: int, n: int, grid: ShardGrid, sub_grid_dimension: int, owner_ptr: int, nranks: int,
                        send_ptr: int, bitmaps_ptr: int, device: int = 0):
    """Route without keys: bitmaps_ptr receives nranks rows of ceil(n/64) u64
    membership words (pcc_shard_route_bitmaps); returns the counts per rank."""
    counts = (C.c_uint64 * nranks)()
    _check(lib().pcc_shard_route_bitmaps(C.c_void_p(pts_ptr), n, C.byref(grid), sub_grid_dimension,
                                         C.c_void_p(owner_ptr), nranks, C.c_void_p(send_ptr), C.c_void_p(bitmaps_ptr),
                                         counts, device))
    return [int(c) for c in counts]


def shard_route_bitmaps_hist(pts_ptr: int, n: int, grid: ShardGrid, sub_grid_dimension: int, owner_ptr: int,
                             nranks: int, hist_ptr: int, send_ptr: int, bitmaps_ptr: int, device: int = 0):
    """One-pass shard_route_bitmaps (pcc_shard_route_bitmaps_hist): hist_ptr =
    this rank's points per unit (same units as the route) over the same points."""
    counts = (C.c_uint64 * nranks)()
    _check(lib().pcc_shard_route_bitmaps_hist(C.c_void_p(pts_ptr), n, C.byref(grid), sub_grid_dimension,
                                              C.c_void_p(owner_ptr), nranks, C.c_void_p(hist_ptr),
                                              C.c_void_p(send_ptr), C.c_void_p(bitmaps_ptr), counts, device))
    return [int(c) for c in counts]


def shard_keys_from_bitmaps(bitmaps_ptr: int, nwords, key0, keys_ptr: int, nkeys: int, device: int = 0):
    """Global keys of received points from the senders' bitmap rows (pcc_shard_keys_from_bitmaps)."""
    ns = len(nwords)
    nw = (C.c_uint64 * ns)(*[int(v) for v in nwords])
    k0 = (C.c_uint64 * ns)(*[int(v) for v in key0])
    _check(lib().pcc_shard_keys_from_bitmaps(C.c_void_p(bitmaps_ptr), nw, k0, ns, C.c_void_p(keys_ptr), nkeys,
                                             device))


def shard_resolve_buckets(seg_n, seg_bucket, nbuckets: int, pts_ptr: int, keys_ptr: int, file_points,
                          batch_size: int, limit: int, kept_ptr: int, sub_pts_ptr: int, sub_keys_ptr: int,
                          device: int = 0):
    """pcc_shard_resolve_buckets: returns (state, spill_batch, kept_n) per bucket
    (numpy) and the row totals (nkept, nsub) written to the device outputs."""
    sn = np.ascontiguousarray(seg_n, dtype=np.uint64).reshape(-1)
    sbk = np.ascontiguousarray(seg_bucket, dtype=np.uint32).reshape(-1)
    fp = np.ascontiguousarray([int(v) for v in file_points], dtype=np.uint64)
    st = np.zeros(nbuckets, np.uint32)
    sb = np.zeros(nbuckets, np.uint32)
    kn = np.zeros(nbuckets, np.uint64)
    nk, ns = C.c_uint64(0), C.c_uint64(0)
    _check(lib().pcc_shard_resolve_buckets(sn.ctypes.data, sbk.ctypes.data, len(sn), nbuckets, C.c_void_p(pts_ptr),
                                           C.c_void_p(keys_ptr), fp.ctypes.data, len(fp), batch_size, limit,
                                           st.ctypes.data, sb.ctypes.data, kn.ctypes.data, C.c_void_p(kept_ptr),
                                           C.c_void_p(sub_pts_ptr), C.c_void_p(sub_keys_ptr), C.byref(nk),
                                           C.byref(ns), device))
    return st, sb, kn, nk.value, ns.value


def shard_lpt(w, world: int):
    """pcc_shard_lpt: (owner per item uint32, load per rank float64)."""
    w = np.ascontiguousarray(w, dtype=np.float64).reshape(-1)
    own = np.zeros(len(w), np.uint32)
    load = np.zeros(world, np.float64)
    _check(lib().pcc_shard_lpt(w.ctypes.data, len(w), world, own.ctypes.data, load.ctypes.data))
    return own, load


def shard_plan_search(whole_w, slab_off, slab_w, child_off, child_w, kmax: int, world: int, owners: bool = False):
    """pcc_shard_plan_search: (best k, its estimate), and with owners=True also
    (whole-cell owners, slab owners, child owners, phase-1 loads, phase-2 loads)
    of the best k's placement."""
    f = lambda a, t: np.ascontiguousarray(a, dtype=t).reshape(-1)
    ww, so, sw, co, cw = (f(whole_w, np.float64), f(slab_off, np.uint64), f(slab_w, np.float64),
                          f(child_off, np.uint64), f(child_w, np.float64))
    bk, bt = C.c_uint32(0), C.c_double(0.0)
    out = None
    if owners:
        out = (np.zeros(len(ww), np.uint32), np.zeros(len(sw), np.uint32), np.zeros(len(cw), np.uint32),
               np.zeros(world, np.float64), np.zeros(world, np.float64))
    ptr = lambda a: a.ctypes.data if (a is not None and len(a)) else None
    _check(lib().pcc_shard_plan_search(ww.ctypes.data, so.ctypes.data, ptr(sw), co.ctypes.data, ptr(cw), len(ww), kmax,
                                       world, C.byref(bk), C.byref(bt), *(ptr(a) for a in (out or (None,) * 5))))
    return (bk.value, bt.value) if not owners else (bk.value, bt.value) + out


def write_cell_view(out_dir: str, view: "CellView"):
    _check(lib().pcc_write_cell_view(out_dir.encode(), C.addressof(view)))


def shard_route(pts_ptr: int, n: int, key0: int, grid: ShardGrid, owner_ptr: int, nranks: int, send_ptr: int,
                keys_ptr: int, device: int = 0):
    counts = (C.c_uint64 * nranks)()
    _check(lib().pcc_shard_route(C.c_void_p(pts_ptr), n, key0, C.byref(grid), C.c_void_p(owner_ptr), nranks,
                                 C.c_void_p(send_ptr), C.c_void_p(keys_ptr), counts, device))
    return [int(c) for c in counts]


def convert_from_paths(paths, output: str, batch_size: int = 10_000, device: int = 0):
    """lib.rs:11-60 convert_from_paths (PLY inputs)."""
    arr = (C.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
    opt = default_options(batch_size=batch_size, device=device)
    _check(lib().pcc_convert_files(os.fsencode(output), arr, len(paths), C.byref(opt)))


def write_ply(path: str, pts: np.ndarray, ascii: bool = False):
    """Binary little-endian (or ASCII) PLY with x,y,z float + red,green,blue,alpha uchar."""
    pts = np.ascontiguousarray(pts, dtype=POINT_DTYPE)
    hdr = ("ply\nformat %s 1.0\nelement vertex %d\nproperty float x\nproperty float y\nproperty float z\n"
           "property uchar red\nproperty uchar green\nproperty uchar blue\nproperty uchar alpha\nend_header\n"
           % ("ascii" if ascii else "binary_little_endian", len(pts)))
    with open(path, "wb") as f:
        f.write(hdr.encode())
        if ascii:
            for p in pts:
                f.write(("%r %r %r %d %d %d %d\n" % (float(p["x"]), float(p["y"]), float(p["z"]), *p["rgba"])).encode())
        else:
            f.write(pts.tobytes())
