"""custom_envs/simple_trap_env: the reference's trap gridworld, stepped on the GPU (envs.TrapEnv).

trap_map.npz holds the reference's walkable bitmap (tile_map.py:40, map.txt) as data."""
