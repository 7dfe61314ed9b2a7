"""Node exporter control plane (``kgs exporter``); the data plane is native C++."""
