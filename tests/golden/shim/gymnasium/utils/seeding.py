import numpy as np

RandomNumberGenerator = np.random.Generator


def np_random(seed=None):
    seed_seq = np.random.SeedSequence(seed)
    rng = RandomNumberGenerator(np.random.PCG64(seed_seq))
    return rng, seed_seq.entropy
