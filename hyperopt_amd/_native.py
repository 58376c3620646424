"""ctypes binding of libtpe_hip.so (declared in include/tpe_hip.h).

The library is built in-tree (``__graft_entry__.build()`` or
``python -m hyperopt_amd.build``).  There is no fallback: if the library is
missing or does not load, every suggest call raises ``NativeUnavailable``.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('TPE_HIP_LIB') or os.path.join(HERE, 'libtpe_hip.so')   # override: A/B builds
ABI_VERSION = 22
FIT_DELTA_MAX = 16             # TPE_FIT_DELTA_MAX: new observations read as a delta (no merge)
BEST_PER_TILE = 8         # TPE_BEST_PER_TILE: tile_best slots per candidate tile

FAM_GAUSS, FAM_LOGGAUSS, FAM_QGAUSS, FAM_QLOGGAUSS, FAM_CATEGORICAL = range(5)
F_HAS_LOW, F_HAS_HIGH, F_POOLED, F_CAT_LAZY, F_NO_TABLE, F_PREFIT, F_FGT, F_REMOTE, F_LOGPOLY = \
    1, 2, 4, 8, 16, 32, 64, 128, 256
TAB_NONE, TAB_CELLS, TAB_LATTICE, TAB_LOGPOLY = 0, 1, 2, 3
TAB_PER_BLOCK = 8                  # include/tpe_hip.h TPE_TAB_PER_BLOCK
TAB_ROW_UNITS = 3                  # include/tpe_hip.h TPE_TAB_ROW_UNITS: 16-B units of a cell row
BATCH_NO_EXPAND, BATCH_WRITE_CAND, BATCH_NO_FUSE, BATCH_ORDERED_DRAWS, BATCH_TAB_EXACT, BATCH_NO_TAB_FAST = \
    1, 2, 4, 8, 16, 32
BATCH_NO_FAST2 = 64
PREC_F32, PREC_F64 = 0, 1

# numpy mirrors of the C structs (the host builds arrays of them and copies
# them to device memory in one transfer)
PROBLEM_DTYPE = np.dtype([
    ('family', '<i4'), ('flags', '<i4'), ('n_cand', '<i4'), ('n_upper', '<i4'),
    ('cand_off', '<i8'), ('cand_base', '<i8'), ('n_cand_global', '<i8'),
    ('n_splits', '<i4'), ('tile_off', '<i4'), ('n_tiles', '<i4'), ('samp_off', '<i4'),
    ('samp_len', '<i4'), ('below_off', '<i4'), ('below_len', '<i4'), ('above_off', '<i4'),
    ('above_len', '<i4'), ('wide_off', '<i4'), ('wide_len', '<i4'), ('grid_off', '<i4'),
    ('grid_n', '<i4'), ('sort_slot', '<i4'),
    ('low', '<f8'), ('high', '<f8'), ('q', '<f8'), ('below_base', '<f8'), ('above_base', '<f8'),
    ('prior_mu', '<f4'), ('prior_a', '<f4'), ('prior_c', '<f4'), ('narrow_cmax', '<f4'),
    ('narrow_amin', '<f4'), ('grid_lo', '<f4'), ('grid_inv', '<f4'),
    ('key_lo', '<f4'), ('key_inv', '<f4'), ('pool_first', '<i4'),
    ('key0', '<u4'), ('key1', '<u4'), ('ctr2', '<u4'), ('ctr3', '<u4'),
    ('tab_mode', '<i4'), ('tab_off', '<i4', (2,)), ('tab_n', '<i4', (2,)), ('tab_lo', '<f4', (2,)),
    ('tab_inv', '<f4', (2,)), ('fgt_a', '<f4'), ('lat_lo', '<i8'), ('fgt_off', '<i4'), ('fgt_n', '<i4'),
    ('fgt_lo', '<f8'),
])
assert PROBLEM_DTYPE.itemsize == 256
TAB_JOB_DTYPE = np.dtype([('problem', '<i4'), ('side', '<i4'), ('kind', '<i4'), ('n', '<i4'), ('off', '<i4'),
                          ('block0', '<i4'), ('rows_off', '<i4'), ('rows_n', '<i4'), ('wide_off', '<i4'),
                          ('wide_n', '<i4'), ('lo', '<f4'), ('inv', '<f4')])
assert TAB_JOB_DTYPE.itemsize == 48
TILE_DTYPE = np.dtype([('problem', '<i4'), ('cand_start', '<i4'), ('work_first', '<i4'), ('n_splits', '<i4')])
WORK_DTYPE = np.dtype([('problem', '<i4'), ('split', '<i4'), ('cand_start', '<i4'),
                       ('k_start', '<i4'), ('k_end', '<i4'), ('n_splits', '<i4')])
BEST_DTYPE = np.dtype([('score', '<f8'), ('l', '<f8'), ('g', '<f8'), ('idx', '<i8')])
FIT_JOB_DTYPE = np.dtype([
    ('obs', '<u8'), ('n_obs', '<i8'), ('seg_off', '<i8'), ('below_off', '<i4'), ('n_below', '<i4'),
    ('family', '<i4'), ('flags', '<i4'), ('lf', '<i4'), ('problem_first', '<i4'), ('n_problems', '<i4'),
    ('above_off', '<i4'), ('wide_off', '<i4'), ('grid_off', '<i4'), ('grid_n', '<i4'), ('reserved', '<i4'),
    ('prior_mu', '<f8'), ('prior_sigma', '<f8'), ('prior_weight', '<f8'), ('low', '<f8'), ('high', '<f8'),
    ('ord_key_in', '<u8'), ('ord_idx_in', '<u8'), ('n_ord_in', '<i8'), ('ord_key_out', '<u8'), ('ord_idx_out', '<u8'),
])
assert FIT_JOB_DTYPE.itemsize == 152
RESULT_DTYPE = np.dtype([('score', '<f8'), ('l', '<f8'), ('g', '<f8'), ('value', '<f8'),
                         ('idx', '<i8'), ('global_idx', '<i8')])
assert RESULT_DTYPE.itemsize == 48


class Batch(ctypes.Structure):
    _fields_ = [
        ('problems', ctypes.c_void_p), ('n_problems', ctypes.c_int32),
        ('precision', ctypes.c_int32), ('sample', ctypes.c_int32), ('sort_end_bit', ctypes.c_int32),
        ('key_bits', ctypes.c_int32), ('flags', ctypes.c_int32),
        ('comp32', ctypes.c_void_p), ('comp64', ctypes.c_void_p), ('samp', ctypes.c_void_p),
        ('grid', ctypes.c_void_p),
        ('cand', ctypes.c_void_p), ('coord', ctypes.c_void_p),
        ('keys', ctypes.c_void_p), ('vals', ctypes.c_void_p),
        ('keys_sorted', ctypes.c_void_p), ('vals_sorted', ctypes.c_void_p),
        ('sort_tmp', ctypes.c_void_p), ('sort_tmp_bytes', ctypes.c_uint64),
        ('total_cand', ctypes.c_int64),
        ('tiles', ctypes.c_void_p), ('n_tiles', ctypes.c_int32), ('n_fin_tiles', ctypes.c_int32),
        ('sort_count', ctypes.c_int64), ('fin_tiles', ctypes.c_void_p),
        ('work', ctypes.c_void_p),
        ('n_work_cont', ctypes.c_int32), ('n_work_qgauss', ctypes.c_int32),
        ('n_work_qlog', ctypes.c_int32), ('fgt_max_boxes', ctypes.c_int32),
        ('part', ctypes.c_void_p), ('l_out', ctypes.c_void_p), ('g_out', ctypes.c_void_p),
        ('tile_best', ctypes.c_void_p), ('result', ctypes.c_void_p),
        ('ce_count', ctypes.c_void_p),
        ('fit', ctypes.c_void_p), ('n_fit', ctypes.c_int32), ('fgt_max_cells', ctypes.c_int32),
        ('below_idx', ctypes.c_void_p), ('fit_seg', ctypes.c_void_p), ('fit_total', ctypes.c_int64),
        ('fit_keys', ctypes.c_void_p), ('fit_keys_sorted', ctypes.c_void_p),
        ('fit_vals', ctypes.c_void_p), ('fit_vals_sorted', ctypes.c_void_p),
        ('fit_max_new', ctypes.c_int64), ('fit_max_obs', ctypes.c_int64), ('fit_max_merge', ctypes.c_int64),
        ('fit_n_delta', ctypes.c_int64),
        ('draw_pref', ctypes.c_void_p), ('draw_blocks', ctypes.c_int64), ('n_sorted', ctypes.c_int32),
        ('tab_fast', ctypes.c_int32), ('pool_best', ctypes.c_void_p),
        ('tab_jobs', ctypes.c_void_p), ('n_tab_jobs', ctypes.c_int32), ('tab_blocks', ctypes.c_int32),
        ('tab', ctypes.c_void_p), ('tab_units', ctypes.c_int64),
        ('samp_tiles', ctypes.c_void_p), ('n_samp_tiles', ctypes.c_int32), ('n_samp_eager', ctypes.c_int32),
        ('tab_tiles', ctypes.c_void_p), ('n_tab_tiles', ctypes.c_int32), ('early_select', ctypes.c_int32),
        ('run_best', ctypes.c_void_p), ('n_late', ctypes.c_int32), ('tiles_per_problem', ctypes.c_int32),
    ]


class LabelIn(ctypes.Structure):
    _fields_ = [
        ('family', ctypes.c_int32), ('flags', ctypes.c_int32), ('upper', ctypes.c_int32),
        ('label_ix', ctypes.c_int32),
        ('low', ctypes.c_double), ('high', ctypes.c_double), ('q', ctypes.c_double),
        ('below_w', ctypes.c_void_p), ('below_mu', ctypes.c_void_p), ('below_sigma', ctypes.c_void_p),
        ('below_k', ctypes.c_int64),
        ('above_w', ctypes.c_void_p), ('above_mu', ctypes.c_void_p), ('above_sigma', ctypes.c_void_p),
        ('above_k', ctypes.c_int64),
        ('ids', ctypes.c_void_p), ('n_ids', ctypes.c_int64),
        ('dev_obs', ctypes.c_void_p), ('n_obs', ctypes.c_int64),
        ('below_idx', ctypes.c_void_p), ('n_below', ctypes.c_int32), ('lf', ctypes.c_int32),
        ('prior_mu', ctypes.c_double), ('prior_sigma', ctypes.c_double), ('prior_weight', ctypes.c_double),
        ('ord_key_in', ctypes.c_void_p), ('ord_idx_in', ctypes.c_void_p), ('n_ord_in', ctypes.c_int64),
        ('ord_key_out', ctypes.c_void_p), ('ord_idx_out', ctypes.c_void_p),
    ]


def _dtype_of(struct):
    """numpy mirror of a ctypes Structure (pointers as uint64): lets a whole
    array of structs be filled with one tuple assignment per element."""
    conv = {ctypes.c_int32: '<i4', ctypes.c_int64: '<i8', ctypes.c_double: '<f8', ctypes.c_void_p: '<u8',
            ctypes.c_uint64: '<u8'}
    names, formats, offsets = [], [], []
    for name, ct in struct._fields_:
        names.append(name)
        formats.append(conv[ct])
        offsets.append(getattr(struct, name).offset)
    return np.dtype(dict(names=names, formats=formats, offsets=offsets, itemsize=ctypes.sizeof(struct)))


LABEL_DTYPE = _dtype_of(LabelIn)


class PackInfo(ctypes.Structure):
    _fields_ = [
        ('off_problems', ctypes.c_int64), ('off_tiles', ctypes.c_int64), ('off_work', ctypes.c_int64),
        ('off_comp32', ctypes.c_int64), ('off_comp64', ctypes.c_int64), ('off_samp', ctypes.c_int64),
        ('off_grid', ctypes.c_int64), ('n_problems', ctypes.c_int64), ('n_tiles', ctypes.c_int64),
        ('n_work_cont', ctypes.c_int32), ('n_work_qgauss', ctypes.c_int32), ('n_work_qlog', ctypes.c_int32),
        ('any_pruned', ctypes.c_int32), ('part_total', ctypes.c_int64), ('blob_bytes', ctypes.c_int64),
        ('key_bits', ctypes.c_int32), ('sort_end_bit', ctypes.c_int32),
        ('off_fit', ctypes.c_int64), ('off_below_idx', ctypes.c_int64), ('off_fit_seg', ctypes.c_int64),
        ('n_fit', ctypes.c_int32), ('fgt_max_boxes', ctypes.c_int32), ('fit_total', ctypes.c_int64),
        ('sort_count', ctypes.c_int64),
        ('off_fin_tiles', ctypes.c_int64), ('n_fin_tiles', ctypes.c_int64), ('fit_max_new', ctypes.c_int64),
        ('fit_max_obs', ctypes.c_int64), ('fit_max_merge', ctypes.c_int64), ('fit_n_delta', ctypes.c_int64),
        ('n_sorted', ctypes.c_int64), ('draw_blocks', ctypes.c_int64), ('n_pooled', ctypes.c_int64),
        ('off_tab_jobs', ctypes.c_int64), ('n_tab_jobs', ctypes.c_int64), ('tab_blocks', ctypes.c_int64),
        ('tab_units', ctypes.c_int64),
        ('off_samp_tiles', ctypes.c_int64), ('n_samp_tiles', ctypes.c_int64), ('n_samp_eager', ctypes.c_int64),
        ('off_tab_tiles', ctypes.c_int64), ('n_tab_tiles', ctypes.c_int64),
        ('off_expand', ctypes.c_int64), ('n_expand', ctypes.c_int64),
        ('fgt_max_cells', ctypes.c_int64),
        ('up_off', ctypes.c_int64 * 4), ('up_len', ctypes.c_int64 * 4), ('n_up', ctypes.c_int32),
        ('pad_', ctypes.c_int32), ('off_patch', ctypes.c_int64),
    ]


class LevelWS(ctypes.Structure):
    """tpe_level_ws: caller-owned buffers of tpe_level_run."""
    _fields_ = [
        ('pinned', ctypes.c_void_p), ('pinned_bytes', ctypes.c_int64), ('pinned_dev', ctypes.c_void_p),
        ('blob', ctypes.c_void_p), ('blob_bytes', ctypes.c_int64),
        ('cand', ctypes.c_void_p), ('coord', ctypes.c_void_p),
        ('keys', ctypes.c_void_p), ('vals', ctypes.c_void_p), ('keys_sorted', ctypes.c_void_p),
        ('vals_sorted', ctypes.c_void_p), ('cand_cap', ctypes.c_int64),
        ('sort_tmp', ctypes.c_void_p), ('sort_tmp_bytes', ctypes.c_int64),
        ('part', ctypes.c_void_p), ('part_cap', ctypes.c_int64),
        ('tile_best', ctypes.c_void_p), ('best_cap', ctypes.c_int64),
        ('result', ctypes.c_void_p), ('result_cap', ctypes.c_int64),
        ('fit_keys', ctypes.c_void_p), ('fit_keys_sorted', ctypes.c_void_p),
        ('fit_vals', ctypes.c_void_p), ('fit_vals_sorted', ctypes.c_void_p), ('fit_cap', ctypes.c_int64),
        ('draw_pref', ctypes.c_void_p), ('draw_pref_cap', ctypes.c_int64),
        ('pool_best', ctypes.c_void_p), ('pool_best_cap', ctypes.c_int64),
        ('tab', ctypes.c_void_p), ('tab_cap', ctypes.c_int64),
    ]


class LevelNeed(ctypes.Structure):
    """tpe_level_need: sizes one level needs."""
    _fields_ = [(k, ctypes.c_int64) for k in ('pinned_bytes', 'blob_bytes', 'cand', 'sort_tmp_bytes', 'part',
                                              'best', 'result', 'fit',
                                              'draw_pref', 'pool_best', 'tab')]


E_HIP = -2
E_SPACE = -4
E_FALLBACK = -5          # tpe_suggest_tree: the space / history needs the general (host) path
TREE_MAX_PARENTS = 4
TREE_NO_SPECULATE = 1 << 8


class TreeLabel(ctypes.Structure):
    """tpe_tree_label: one hyperparameter of a tree space (tpe_suggest_tree)."""
    _fields_ = [
        ('family', ctypes.c_int32), ('flags', ctypes.c_int32), ('upper', ctypes.c_int32),
        ('label_ix', ctypes.c_int32),
        ('low', ctypes.c_double), ('high', ctypes.c_double), ('prior_mu', ctypes.c_double),
        ('prior_sigma', ctypes.c_double),
        ('p_prior', ctypes.c_void_p), ('tids', ctypes.c_void_p), ('values', ctypes.c_void_p),
        ('order', ctypes.c_void_p), ('n_obs', ctypes.c_int64),
        ('depth', ctypes.c_int32), ('n_parents', ctypes.c_int32),
        ('parent', ctypes.c_int32 * TREE_MAX_PARENTS), ('parent_cat', ctypes.c_int32 * TREE_MAX_PARENTS),
        ('q', ctypes.c_double),
        ('host_w', ctypes.c_void_p * 2), ('host_mu', ctypes.c_void_p * 2), ('host_sigma', ctypes.c_void_p * 2),
        ('host_k', ctypes.c_int64 * 2),
        ('dev_obs', ctypes.c_void_p), ('ord_key_in', ctypes.c_void_p), ('ord_idx_in', ctypes.c_void_p),
        ('n_ord_in', ctypes.c_int64), ('ord_key_out', ctypes.c_void_p), ('ord_idx_out', ctypes.c_void_p),
        ('side_order', ctypes.c_void_p * 2), ('side_n', ctypes.c_int64 * 2),
    ]


COMM_ID_BYTES = 128          # TPE_COMM_ID_BYTES
EXCHANGE_HEADER = 64         # TPE_EXCHANGE_HEADER
GATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p)


class Exchange(ctypes.Structure):
    """tpe_exchange: the candidate-shard exchange of a sharded tpe_suggest_tree."""
    _fields_ = [
        ('rank', ctypes.c_int32), ('world', ctypes.c_int32), ('comm', ctypes.c_void_p),
        ('gather', GATHER_FN), ('ctx', ctypes.c_void_p), ('dev', ctypes.c_void_p), ('dev_bytes', ctypes.c_int64),
        ('always', ctypes.c_int32), ('reserved', ctypes.c_int32),
    ]


TREE_LABEL_DTYPE = np.dtype(dict(
    names=[f for f, _ in TreeLabel._fields_],
    formats=['<i4', '<i4', '<i4', '<i4', '<f8', '<f8', '<f8', '<f8', '<u8', '<u8', '<u8', '<u8', '<i8', '<i4', '<i4',
             ('<i4', (TREE_MAX_PARENTS,)), ('<i4', (TREE_MAX_PARENTS,)), '<f8', ('<u8', (2,)), ('<u8', (2,)),
             ('<u8', (2,)), ('<i8', (2,)), '<u8', '<u8', '<u8', '<i8', '<u8', '<u8', ('<u8', (2,)), ('<i8', (2,))],
    offsets=[getattr(TreeLabel, f).offset for f, _ in TreeLabel._fields_], itemsize=ctypes.sizeof(TreeLabel)))

EXPORTS = ('tpe_abi_version', 'tpe_last_error', 'tpe_device_count', 'tpe_tile_size', 'tpe_pinned_device_address',
           'tpe_sort_workspace_bytes', 'tpe_run_batch', 'tpe_fit_above', 'tpe_tables',
           'tpe_sample', 'tpe_sort', 'tpe_score_above', 'tpe_finalize', 'tpe_select', 'tpe_host_fit_parzen', 'tpe_host_fit_split',
           'tpe_host_cat_probs', 'tpe_host_cat_split', 'tpe_host_pack_level', 'tpe_level_run',
           'tpe_replay_mixture', 'tpe_replay_categorical', 'tpe_level_profile', 'tpe_level_profile_read',
           'tpe_suggest_tree', 'tpe_comm_unique_id', 'tpe_comm_init', 'tpe_comm_destroy', 'tpe_combine_results',
           'tpe_host_threads', 'tpe_host_phases', 'tpe_exchange_allgather', 'tpe_debug_fast_lg',
           'tpe_collectives_issued', 'tpe_scatter_f64', 'tpe_move_ranges')

# host phases of tpe_suggest_tree (tpe_host_phases order)
PHASES = ('prefit', 'pack', 'launched', 'synced', 'level', 'return', 'recs')

# tpe_level_run stages (tpe_level_profile_read order)
STAGES = ('fit', 'k_tables', 'k_sample', 'sort', 'above', 'k_finalize', 'k_select')


class StageProf(ctypes.Structure):
    """tpe_stage_prof: one stage of the last profiled tpe_level_run."""
    _fields_ = [('ms', ctypes.c_double), ('units', ctypes.c_double), ('ce', ctypes.c_double),
                ('launches', ctypes.c_int32), ('kernel_ns', ctypes.c_int32)]


class MTState(ctypes.Structure):
    """tpe_mt_state: numpy's legacy RandomState (MT19937 key, position and the
    cached polar-method gauss)."""
    _fields_ = [('key', ctypes.c_uint32 * 624), ('pos', ctypes.c_int32), ('has_gauss', ctypes.c_int32),
                ('gauss', ctypes.c_double)]


class NativeUnavailable(RuntimeError):
    """libtpe_hip.so is missing, fails to load, or finds no HIP device."""


_LIB = None


def load(path=LIB_PATH):
    """Load (once) and type the C-ABI.  Raises NativeUnavailable, never falls back."""
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(path):
        raise NativeUnavailable('%s is not built (run __graft_entry__.build() or '
                                'python -m hyperopt_amd.build)' % path)
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:
        raise NativeUnavailable('cannot load %s: %s' % (path, e))
    lib.tpe_abi_version.restype = ctypes.c_int
    lib.tpe_last_error.restype = ctypes.c_char_p
    lib.tpe_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    lib.tpe_tile_size.restype = ctypes.c_int
    lib.tpe_pinned_device_address.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]
    lib.tpe_pinned_device_address.restype = ctypes.c_int
    lib.tpe_sort_workspace_bytes.argtypes = [ctypes.c_int64, ctypes.POINTER(ctypes.c_uint64)]
    lib.tpe_sort_workspace_bytes.restype = ctypes.c_int
    for name in ('tpe_run_batch', 'tpe_fit_above', 'tpe_tables', 'tpe_sample', 'tpe_sort', 'tpe_score_above', 'tpe_finalize', 'tpe_select'):
        fn = getattr(lib, name)
        fn.argtypes = [ctypes.POINTER(Batch), ctypes.c_void_p]
        fn.restype = ctypes.c_int
    P = ctypes.c_void_p
    lib.tpe_host_fit_parzen.argtypes = [P, ctypes.c_int64, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                        ctypes.c_int32, P, P, P]
    lib.tpe_host_fit_parzen.restype = ctypes.c_int64
    D = ctypes.c_double
    lib.tpe_host_fit_split.argtypes = [P, P, P, ctypes.c_int64, P, ctypes.c_int64, D, D, D, ctypes.c_int32, P, P]
    lib.tpe_host_fit_split.restype = ctypes.c_int
    lib.tpe_host_cat_probs.argtypes = [P, ctypes.c_int64, ctypes.c_int32, P, ctypes.c_double, ctypes.c_int32, P]
    lib.tpe_host_cat_probs.restype = ctypes.c_int
    lib.tpe_host_cat_split.argtypes = [P, P, ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int32, P, D, ctypes.c_int32,
                                       P, P]
    lib.tpe_host_cat_split.restype = ctypes.c_int
    I64 = ctypes.c_int64
    lib.tpe_replay_mixture.argtypes = [P, P, P, P, I64, ctypes.c_int32, D, D, I64, P]
    lib.tpe_replay_mixture.restype = ctypes.c_int
    lib.tpe_replay_categorical.argtypes = [P, P, I64, I64, P]
    lib.tpe_replay_categorical.restype = ctypes.c_int
    lib.tpe_host_pack_level.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                        ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, P, ctypes.c_int64,
                                        ctypes.POINTER(PackInfo)]
    lib.tpe_host_pack_level.restype = ctypes.c_int
    lib.tpe_level_run.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64,
                                  ctypes.c_int64, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(LevelWS),
                                  ctypes.POINTER(LevelNeed), P, P]
    lib.tpe_level_run.restype = ctypes.c_int
    I32 = ctypes.c_int32
    lib.tpe_suggest_tree.argtypes = [P, I32, P, I64, D, I32, P, I32, I32, I64, I64, ctypes.POINTER(Exchange),
                                     ctypes.c_uint64, D, I64, I32,
                                     ctypes.POINTER(LevelWS), ctypes.POINTER(LevelNeed), P, P, P, P, P]
    lib.tpe_suggest_tree.restype = ctypes.c_int
    lib.tpe_comm_unique_id.argtypes = [P]
    lib.tpe_comm_unique_id.restype = ctypes.c_int
    lib.tpe_comm_init.argtypes = [I32, I32, P, I32, ctypes.POINTER(ctypes.c_void_p)]
    lib.tpe_comm_init.restype = ctypes.c_int
    lib.tpe_comm_destroy.argtypes = [P]
    lib.tpe_comm_destroy.restype = ctypes.c_int
    lib.tpe_combine_results.argtypes = [P, I32, I64, P]
    lib.tpe_combine_results.restype = ctypes.c_int
    lib.tpe_exchange_allgather.argtypes = [ctypes.POINTER(Exchange), P, I64, P, P]
    lib.tpe_exchange_allgather.restype = ctypes.c_int
    lib.tpe_host_threads.argtypes = [I32, ctypes.POINTER(I32)]
    lib.tpe_host_threads.restype = ctypes.c_int
    lib.tpe_host_phases.argtypes = [I32, P, I32]
    lib.tpe_host_phases.restype = ctypes.c_int
    lib.tpe_debug_fast_lg.argtypes = [P, I64]
    lib.tpe_debug_fast_lg.restype = ctypes.c_int
    lib.tpe_collectives_issued.argtypes = [ctypes.POINTER(I64)]
    lib.tpe_collectives_issued.restype = ctypes.c_int
    lib.tpe_scatter_f64.argtypes = [P, I64, P, P]
    lib.tpe_scatter_f64.restype = ctypes.c_int
    lib.tpe_move_ranges.argtypes = [P, ctypes.c_int32, ctypes.c_int32, P, P, P]
    lib.tpe_move_ranges.restype = ctypes.c_int
    lib.tpe_level_profile.argtypes = [ctypes.c_int32]
    lib.tpe_level_profile.restype = ctypes.c_int
    lib.tpe_level_profile_read.argtypes = [ctypes.POINTER(StageProf), ctypes.c_int32]
    lib.tpe_level_profile_read.restype = ctypes.c_int
    if lib.tpe_abi_version() != ABI_VERSION:
        raise NativeUnavailable('ABI mismatch: library %d, bindings %d' % (lib.tpe_abi_version(), ABI_VERSION))
    _LIB = lib
    return lib


def check(rc, lib, what):
    if rc != 0:
        msg = lib.tpe_last_error().decode(errors='replace')
        raise RuntimeError('%s failed (%d): %s' % (what, rc, msg))


def tile_size():
    return load().tpe_tile_size()


def collectives_issued(lib=None):
    """ncclAllGather calls the library has issued in this process
    (tpe_collectives_issued)."""
    lib = lib or load()
    n = ctypes.c_int64(0)
    check(lib.tpe_collectives_issued(ctypes.byref(n)), lib, 'tpe_collectives_issued')
    return int(n.value)
