"""GPU/PID → Kubernetes pod attribution (kubelet pod-resources gRPC + cgroups)."""
