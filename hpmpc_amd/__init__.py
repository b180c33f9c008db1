"""hpmpc_amd -- MI355X-native backward Riccati recursion + interior-point MPC hot path (HPMPC drop-in)."""
