"""Plugin signals (laser/plugin/signals.py:1-22): raised by hooks to skip a state
or to keep a world state out of open_states."""


class PluginSignal(Exception):
    pass


class PluginSkipWorldState(PluginSignal):
    """Raised by an add_world_state hook: the world state is not added."""


class PluginSkipState(PluginSignal):
    """Raised by an execute_state / pre / post hook: the state is dropped."""
