set -u
export PYTHONUNBUFFERED=1
timeout -k 10 200 python scripts/wgrad_probe.py
echo PLAIN; TFX_WGRAD_PLAIN_PROBE=1 timeout -k 10 200 python scripts/wgrad_probe.py
