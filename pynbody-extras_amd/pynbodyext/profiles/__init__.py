"""pynbodyext.profiles — radial profiles binned and reduced on MI355X.

Same exports as the reference (pynbodyext/profiles/__init__.py:4-9) minus
StarAgeProfile, which bins by stellar age and is off the hot path.
"""
from .base import ProfileBuilderBase, RadialProfileBuilder
from .bins import BinsSet
from .profile import Profile, ProfileBase, SubProfile
from .proarray import ProfileArray, StatisticBase
from .spatial_profile import RadialProfile

__all__ = ["RadialProfileBuilder", "ProfileBuilderBase", "Profile", "ProfileBase", "SubProfile",
           "RadialProfile", "BinsSet", "ProfileArray", "StatisticBase"]
