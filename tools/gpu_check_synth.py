"""GPU: device generator bytes == host generator bytes (small spec)."""
import sys
from pathlib import Path
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from gfa2network_amd import synth
for spec in [(10, 20, 0, True), (1000, 5000, 3, False), (123457, 400000, 7, True)]:
    h = synth.host_bytes(spec[0], spec[1], seed=spec[2], rc_tag=spec[3])
    d = synth.DeviceInput(spec[0], spec[1], seed=spec[2], rc_tag=spec[3]).download()
    assert h == d, spec
print("synth host==device OK")
