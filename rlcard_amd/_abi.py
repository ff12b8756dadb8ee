"""ctypes binding of the C ABI (include/cardsim.h) to the in-tree HIP engine rlcard_amd/libcardsim.so.

There is no CPU fallback: if the library is missing, or no GPU is visible, calls raise.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, os.environ.get('CARDSIM_LIB', 'libcardsim.so'))   # CARDSIM_LIB: A/B builds only

GAME_IDS = {'blackjack': 0, 'leduc-holdem': 1, 'limit-holdem': 2, 'doudizhu': 3, 'no-limit-holdem': 4}

CS_OK = 0
_ERRORS = {-1: 'CS_E_INVALID', -2: 'CS_E_DEVICE', -3: 'CS_E_STATE', -4: 'CS_E_UNSUPPORTED'}


class Config(C.Structure):
    _fields_ = [('num_players', C.c_int32), ('num_decks', C.c_int32), ('chips_for_each', C.c_int32),
                ('dealer_plus1', C.c_int32), ('rng_mode', C.c_int32), ('reserved', C.c_int32 * 3)]


RNG_MODES = {'mt19937': 0, 'philox': 1}   # cs_config.rng_mode


class GameInfo(C.Structure):
    _fields_ = [('obs_dim', C.c_int32), ('num_actions', C.c_int32), ('num_players', C.c_int32),
                ('legal_bytes', C.c_int32), ('action_bytes', C.c_int32), ('state_words', C.c_int32),
                ('action_feature_dim', C.c_int32), ('rng_period', C.c_int32), ('game_words', C.c_int32),
                ('deal_queue_depth', C.c_int32), ('envs_per_wave', C.c_int32)]


ABI_VERSION = 2   # the cs_game_info layout above: CS_ABI_VERSION 2 (3 keeps it and adds the cs_state_* functions)


class StepOut(C.Structure):
    _fields_ = [('obs', C.c_void_p), ('legal', C.c_void_p), ('player', C.c_void_p), ('reward', C.c_void_p),
                ('done', C.c_void_p)]


class TrajOut(C.Structure):
    _fields_ = [('obs', C.c_void_p), ('legal', C.c_void_p), ('player', C.c_void_p), ('action', C.c_void_p),
                ('reward', C.c_void_p), ('done', C.c_void_p), ('final_obs', C.c_void_p)]


class TransOut(C.Structure):
    _fields_ = [('next_t', C.c_void_p), ('end_t', C.c_void_p), ('reward', C.c_void_p), ('done', C.c_void_p),
                ('ret', C.c_void_p)]


class DmcBatch(C.Structure):
    _fields_ = [('state', C.c_void_p), ('action', C.c_void_p), ('target', C.c_void_p), ('done', C.c_void_p),
                ('episode_return', C.c_void_p)]


# every symbol include/cardsim.h declares (tests check the library exports all of them)
SYMBOLS = ('cs_game_info_get', 'cs_create', 'cs_destroy', 'cs_seed', 'cs_reset', 'cs_step', 'cs_observe',
           'cs_rollout', 'cs_traj_probe', 'cs_transitions', 'cs_legal_lists', 'cs_action_features', 'cs_get_env_state',
           'cs_set_env_state', 'cs_copy_env_state', 'cs_set_step_record', 'cs_env_rng_words', 'cs_copy_env_rng',
           'cs_load_env_rng', 'cs_get_rng_ctl', 'cs_cfr_train', 'cs_debug_holdem_rank7', 'cs_debug_ddz_legal',
           'cs_debug_set_serial_refill', 'cs_debug_set_kernel_flags',
           'cs_dmc_create', 'cs_dmc_destroy', 'cs_dmc_fill', 'cs_dmc_gather', 'cs_dmc_status', 'cs_dmc_layer1',
           'cs_dmc_select', 'cs_last_error', 'cs_version', 'cs_abi_version', 'cs_state_bytes', 'cs_state_save',
           'cs_state_load')
# symbols an older library build may lack (A/B builds loaded with CARDSIM_LIB); callers check hasattr(lib(), name)
OPTIONAL = ('cs_traj_probe', 'cs_state_bytes', 'cs_state_save', 'cs_state_load')

_lib = None


class CardsimError(RuntimeError):
    pass


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CardsimError('HIP engine not built: %s is missing (run __graft_entry__.build() or '
                           'make -C rlcard_amd/csrc)' % LIB_PATH)
    L = C.CDLL(LIB_PATH)
    vp, i32, i64, u64 = C.c_void_p, C.c_int32, C.c_int64, C.c_uint64
    L.cs_game_info_get.argtypes = [i32, C.POINTER(Config), C.POINTER(GameInfo)]
    L.cs_create.argtypes = [C.POINTER(vp), i32, i64, i32, C.POINTER(Config)]
    L.cs_destroy.argtypes = [vp]
    L.cs_destroy.restype = None
    L.cs_seed.argtypes = [vp, vp, vp, i64, i64, vp]
    L.cs_reset.argtypes = [vp, C.POINTER(StepOut), vp]
    L.cs_step.argtypes = [vp, vp, C.POINTER(StepOut), vp]
    L.cs_observe.argtypes = [vp, i32, C.POINTER(StepOut), vp]
    L.cs_rollout.argtypes = [vp, i32, u64, u64, u64, C.POINTER(TrajOut), vp]
    if hasattr(L, 'cs_traj_probe'):   # (older A/B builds lack it)
        L.cs_traj_probe.argtypes = [vp, i32, C.POINTER(TrajOut), vp]
    if hasattr(L, 'cs_state_bytes'):  # (ABI version 3)
        L.cs_state_bytes.argtypes = [vp, vp]
        L.cs_state_save.argtypes = [vp, vp, vp]
        L.cs_state_load.argtypes = [vp, vp, vp]
    L.cs_transitions.argtypes = [vp, i32, C.POINTER(TrajOut), C.POINTER(TransOut), vp]
    L.cs_legal_lists.argtypes = [vp, vp, i64, vp, vp, vp, vp]
    L.cs_action_features.argtypes = [vp, vp, i64, vp, vp]
    L.cs_get_env_state.argtypes = [vp, i64, vp, i32]
    L.cs_set_env_state.argtypes = [vp, i64, vp, i32]
    L.cs_copy_env_state.argtypes = [vp, i64, vp, vp]
    L.cs_set_step_record.argtypes = [vp, i64, vp, vp]
    L.cs_env_rng_words.argtypes = [vp, vp]
    L.cs_copy_env_rng.argtypes = [vp, i64, vp, vp]
    L.cs_load_env_rng.argtypes = [vp, i64, vp, vp]
    L.cs_get_rng_ctl.argtypes = [vp, i64, vp]
    L.cs_cfr_train.argtypes = [vp, i32, i64, vp, vp, vp, vp, vp]
    L.cs_debug_holdem_rank7.argtypes = [vp, i64, vp, vp]
    L.cs_debug_ddz_legal.argtypes = [vp, vp, vp, i64, vp, vp]
    L.cs_debug_set_serial_refill.argtypes = [vp, i32]
    L.cs_debug_set_kernel_flags.argtypes = [vp, i32]
    L.cs_dmc_create.argtypes = [vp, i32, i32, C.POINTER(vp)]
    L.cs_dmc_destroy.argtypes = [vp]
    L.cs_dmc_destroy.restype = None
    L.cs_dmc_fill.argtypes = [vp, i32, C.POINTER(TrajOut), vp, i64, vp, vp]
    L.cs_dmc_gather.argtypes = [vp, i32, vp, i64, C.POINTER(DmcBatch), vp]
    L.cs_dmc_status.argtypes = [vp, vp]
    L.cs_dmc_layer1.argtypes = [vp, vp, vp, vp, i64, i32, vp, vp, vp, vp]
    L.cs_dmc_select.argtypes = [vp, vp, vp, vp, i64, C.c_float, u64, u64, u64, vp, vp]
    L.cs_last_error.restype = C.c_char_p
    L.cs_version.restype = C.c_char_p
    if hasattr(L, 'cs_abi_version'):   # (older A/B builds lack it)
        L.cs_abi_version.restype = C.c_int32
        if L.cs_abi_version() < ABI_VERSION:
            raise CardsimError('%s implements ABI version %d, this binding needs %d' % (LIB_PATH, L.cs_abi_version(),
                                                                                     ABI_VERSION))
    for name in SYMBOLS:
        if name not in ('cs_destroy', 'cs_dmc_destroy', 'cs_last_error', 'cs_version', 'cs_abi_version'):
            if name in OPTIONAL and not hasattr(L, name):   # older A/B builds (CARDSIM_LIB) lack it
                continue
            getattr(L, name).restype = C.c_int
    _lib = L
    return L


def check(code, what=''):
    if code != CS_OK:
        msg = lib().cs_last_error().decode(errors='replace')
        raise CardsimError('%s failed (%s): %s' % (what, _ERRORS.get(code, code), msg))


def game_info(game, num_players=0, num_decks=-1, chips_for_each=0, dealer_id=None, rng_mode='mt19937'):
    cfg = Config(num_players, num_decks, chips_for_each, 0 if dealer_id is None else int(dealer_id) + 1,
                 RNG_MODES[rng_mode])
    info = GameInfo()
    check(lib().cs_game_info_get(GAME_IDS[game] if isinstance(game, str) else game, C.byref(cfg), C.byref(info)),
          'cs_game_info_get')
    return info, cfg
