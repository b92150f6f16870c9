# Round-4 measurement session h (after the constant-address-space change), part A (final tree): the whole GPU suite and smoke().
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_r4h.log 2>&1 && \
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4h.log 2>&1
