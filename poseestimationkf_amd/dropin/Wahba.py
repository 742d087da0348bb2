"""Drop-in for the reference module ``Wahba`` (Python Kalman Filter/Wahba.py).

Same class, attribute and method names and return types; every computation runs in the
gfx950 kernels of libpekf.so (k_wahba, k_r2q) through the C ABI.  The SVD of the rank-2
attitude profile matrix is replaced by its closed form (DESIGN.md "Wahba closed form");
the rotation is unique, so results agree with np.linalg.svd to rounding.  ``solve`` is an alias
of ``getQuarternion`` (the north_star's name).
"""
from _bootstrap import engine as _eng
from _bootstrap import fastcall as _fc


class Wahba:
    def __init__(self, acc, mag):                       # Wahba.py:4-6
        self.w_initial_acc = acc
        self.w_initial_mag = mag

    def getRotation(self, acc, mag, k_acc, k_mag):      # Wahba.py:8-17
        return _eng.wahba_rotation(self.w_initial_acc, self.w_initial_mag, acc, mag, k_acc, k_mag)[0]

    @staticmethod
    def RotationMatrix2Quart(M):                        # Wahba.py:19-47
        return _eng.rotmat_to_quat(M)[0]

    def getQuarternion(self, acc, mag, k_acc, k_mag):   # Wahba.py:49-50
        return _fc.wahba_quaternion(self.w_initial_acc, self.w_initial_mag, acc, mag, k_acc, k_mag)

    solve = getQuarternion                              # the north_star's name for Wahba.py:49
