"""Runtime helpers: host->device step feeder and HIP-graph capture of the train step."""
