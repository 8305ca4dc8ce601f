"""MI355X-native vectorised RL environment (Gogoro / Thormang) behind the IsaacGymEnvs VecTask API."""
