# compare ranks across two builds of libgpdla (current vs tools/v2lib)
import sys, numpy as np
sys.path.insert(0, '.')
from gp_dla_detection_amd import _lib as L
if len(sys.argv) > 2 and sys.argv[2] == 'v2':
    from pathlib import Path
    L.LIB_PATH = Path('tools/v2lib/libgpdla.so').resolve()
from gp_dla_detection_amd import synthetic as syn
from gp_dla_detection_amd.engine import Engine
from gp_dla_detection_amd.parameters import set_parameters
k = int(sys.argv[1])
model = syn.make_model(k=k, seed=k)
samples = syn.make_samples(70)
spectra = syn.make_dr12q_like_spectra(model, 2, seed=k, mask_fraction=0.05)
with Engine(model, samples, set_parameters(k=k)) as eng:
    out = eng.process(syn.pack_spectra(spectra))
np.save(f'gpurun_out/cmp_{k}_{sys.argv[2] if len(sys.argv)>2 else "cur"}.npy', out['sample_log_likelihoods_dla'])
print(k, out['log_likelihoods_no_dla'], out['sample_log_likelihoods_dla'][0, :5])
