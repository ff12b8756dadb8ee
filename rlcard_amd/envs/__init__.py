"""rlcard's env registry (rlcard/envs/registration.py:8-89 + envs/__init__.py) for the engine's five games."""
import importlib

DEFAULT_CONFIG = {'allow_step_back': False, 'seed': None}


class EnvSpec(object):
    def __init__(self, env_id, entry_point):
        self.env_id = env_id
        mod_name, class_name = entry_point.split(':')
        self._entry_point = getattr(importlib.import_module(mod_name), class_name)

    def make(self, config=DEFAULT_CONFIG):
        return self._entry_point(config)


class EnvRegistry(object):
    def __init__(self):
        self.env_specs = {}

    def register(self, env_id, entry_point):
        if env_id in self.env_specs:
            raise ValueError('Cannot re-register env_id: {}'.format(env_id))
        self.env_specs[env_id] = EnvSpec(env_id, entry_point)

    def make(self, env_id, config=DEFAULT_CONFIG):
        if env_id not in self.env_specs:
            raise ValueError('Cannot find env_id: {}'.format(env_id))
        return self.env_specs[env_id].make(config)


registry = EnvRegistry()


def register(env_id, entry_point):
    return registry.register(env_id, entry_point)


def make(env_id, config={}):
    """rlcard.make(env_id, config): config keys 'seed', 'allow_step_back', the game's 'game_*' keys, and (engine
    only) 'device', the GPU the env lives on."""
    _config = DEFAULT_CONFIG.copy()
    for key in config:
        _config[key] = config[key]
    return registry.make(env_id, _config)


register('blackjack', 'rlcard_amd.envs.blackjack:BlackjackEnv')
register('leduc-holdem', 'rlcard_amd.envs.leducholdem:LeducholdemEnv')
register('limit-holdem', 'rlcard_amd.envs.limitholdem:LimitholdemEnv')
register('doudizhu', 'rlcard_amd.envs.doudizhu:DoudizhuEnv')
register('no-limit-holdem', 'rlcard_amd.envs.nolimitholdem:NolimitholdemEnv')
