"""pybulletgym_amd: MI355X-native batched stepper for the roboschool locomotion envs of
josiahls/pybullet-gym.  Import as ``import pybulletgym_amd``."""
