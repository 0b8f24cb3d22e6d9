"""Noise bookkeeping of the AES drivers, without a GPU (tae_aes_noise_schedule_check).

The reference's BitCt tracks a squared noise level plus the set of fresh-ciphertext ids it is built
from, and panics when an XOR adds two ciphertexts that share an id ("noise components not
independent", src/tfhe/shortint_woppbs_1bit.rs:63-78) or when the level passes MaxNoiseLevel.  The
product validates each driver's round function statically, before any device work; here that is
compared with a line-by-line Python transcription of the reference's code paths:

- fhe_sbox_pbs (src/aes_128/fhe/fhe_sbox_pbs.rs:33-121) over the 1-bit model -- the combination
  whose reference tests are #[ignore]d "since cipher text noise is not independent in calculations"
  (fhe_impls/shortint_woppbs_1bit.rs:160-176): the first MixColumns must fail, a 1-round run pass;
- fhe_sbox_gal_mul_pbs (fhe_sbox_gal_mul_pbs.rs:84-132): passes for every round count at lvl_64
  (test_light_gal_mul / test_full_gal_mul are the reference's green tests);
- the 8-bit model (additive shortint NoiseLevel, MaxNoiseLevel 11): passes.
"""
import itertools

import pytest

import tfhe_aes
from tfhe_aes import _native as N
from tfhe_aes import aes_128

_ids = itertools.count()


class NoiseLevelWithComponents:
    """shortint_woppbs_1bit.rs:34-78"""

    def __init__(self, level, components):
        self.level, self.components = level, set(components)

    @classmethod
    def fresh(cls, level):
        return cls(level, {next(_ids)})

    @classmethod
    def trivial(cls):
        return cls(0, ())

    def copy(self):
        return NoiseLevelWithComponents(self.level, self.components)

    def add_assign(self, rhs, max_sq):
        if self.components & rhs.components:
            raise tfhe_aes.NoiseNotIndependent(N.TAE_E_INDEP, "noise components not independent")
        self.components |= rhs.components
        self.level += rhs.level
        if self.level > max_sq:
            raise tfhe_aes.NoiseTooBig(N.TAE_E_NOISE, f"NoiseTooBig {self.level} > {max_sq}")


def _xor_bytes(a, b, max_sq):  # Byte ^ &Byte: bit by bit
    for x, y in zip(a, b):
        x.add_assign(y, max_sq)
    return a


def _gf_256_mul(a, b, max_sq):
    """fhe_sbox_pbs.rs:33-53 (MSB-first bits; Byte::shl_assign_1 = data_model.rs:45-49)."""
    a = [x.copy() for x in a]
    res = [NoiseLevelWithComponents.trivial() for _ in range(8)]
    for _ in range(8):
        if b & 1:
            _xor_bytes(res, a, max_sq)
        reduce_x8 = a[0]
        a = a[1:] + [NoiseLevelWithComponents.trivial()]
        for i in (3, 4, 6, 7):
            a[i].add_assign(reduce_x8, max_sq)
        b >>= 1
    return res


def sbox_pbs_1bit_schedule(rounds, max_sq):
    """fhe_sbox_pbs::encrypt_block_for_rounds (:75-121) with fresh inputs; SubBytes outputs carry
    noise^2 = 8 (circuit_bootstrap of 8 input bits, shortint_woppbs_1bit.rs:322-325)."""
    F = NoiseLevelWithComponents.fresh
    ek = [[[F(1) for _ in range(8)] for _ in range(4)] for _ in range(44)]
    state = [[[F(1) for _ in range(8)] for _ in range(4)] for _ in range(4)]  # state[r][c]

    def xor_state(words):
        for c in range(4):
            for r in range(4):
                _xor_bytes(state[r][c], words[c][r], max_sq)

    def sub_bytes_shift_rows():
        for r in range(4):
            row = [[F(8) for _ in range(8)] for _ in range(4)]
            state[r] = row[r:] + row[:r]

    xor_state(ek[0:4])
    for i in range(1, rounds):
        sub_bytes_shift_rows()
        cols = []
        for c in range(4):
            col = [state[r][c] for r in range(4)]
            out = []
            for r in range(4):
                v = _gf_256_mul(col[r], 2, max_sq)
                for src, m in (((r - 1) % 4, 1), ((r - 2) % 4, 1), ((r - 3) % 4, 3)):
                    _xor_bytes(v, _gf_256_mul(col[src], m, max_sq), max_sq)
                out.append(v)
            cols.append(out)
        for c in range(4):
            for r in range(4):
                state[r][c] = cols[c][r]
        xor_state(ek[4 * i:4 * i + 4])
    sub_bytes_shift_rows()
    xor_state(ek[40:44])


def _product(param_set, driver, rounds):
    try:
        aes_128.noise_schedule_check(param_set, driver, rounds)
        return None
    except tfhe_aes.TaeError as e:
        return type(e)


def _restated(rounds, max_sq):
    try:
        sbox_pbs_1bit_schedule(rounds, max_sq)
        return None
    except tfhe_aes.TaeError as e:
        return type(e)


@pytest.mark.parametrize("param_set", [N.PARAMS_SQRD_LVL_64, N.PARAMS_SQRD_LVL_256])
@pytest.mark.parametrize("rounds", range(1, 11))
def test_sbox_pbs_1bit_schedule_matches_restatement(param_set, rounds):
    max_sq = tfhe_aes.get_params(param_set)["max_noise_sq"]
    want = _restated(rounds, max_sq)
    assert _product(param_set, N.TAE_DRIVER_SBOX_PBS, rounds) is want
    # the reference's verdict: only the MixColumns-free 1-round run survives
    assert want is (None if rounds == 1 else tfhe_aes.NoiseNotIndependent)


def test_gf_256_mul_alone_breaks_independence():
    """The failing XOR is inside gf_256_mul itself, for every multiplier MixColumns uses."""
    for b in (1, 2, 3):
        with pytest.raises(tfhe_aes.NoiseNotIndependent):
            _gf_256_mul([NoiseLevelWithComponents.fresh(8) for _ in range(8)], b, 64)
    # trivial inputs carry no ids and pass (Byte::trivial in gf_256_mul's own result)
    _gf_256_mul([NoiseLevelWithComponents.trivial() for _ in range(8)], 3, 64)


@pytest.mark.parametrize("rounds", [1, 2, 10])
def test_gal_mul_and_8bit_schedules_pass(rounds):
    assert _product(N.PARAMS_SQRD_LVL_64, N.TAE_DRIVER_GAL_MUL, rounds) is None
    assert _product(N.PARAMS_WOPPBS_8BIT, N.TAE_DRIVER_SBOX_PBS, rounds) is None
    assert _product(N.PARAMS_WOPPBS_8BIT, N.TAE_DRIVER_GAL_MUL, rounds) is None  # the 8-bit model has one driver


def test_schedule_check_arguments():
    with pytest.raises(tfhe_aes.TaeError):
        aes_128.noise_schedule_check(N.PARAMS_SQRD_LVL_64, 7, 1)
    with pytest.raises(tfhe_aes.TaeError):
        aes_128.noise_schedule_check(N.PARAMS_SQRD_LVL_64, N.TAE_DRIVER_GAL_MUL, 0)
    with pytest.raises(tfhe_aes.TaeError):
        aes_128.noise_schedule_check(99, N.TAE_DRIVER_GAL_MUL, 1)
