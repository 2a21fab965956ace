"""Host-side mirror of the reference's ``mtrl`` interface for the MTSAC path.

Same module paths, class names, constructor fields and call conventions as
reginald-mclean/mtrl (``mtrl.config.*``, ``mtrl.rl.algorithms``, ``mtrl.rl.buffers``,
``mtrl.envs``, ``mtrl.experiment``) so ``experiments/mt10_mtmhsac.py`` and
``experiments/mt50_mtmhsac_v2.py`` run unchanged on top of ``libmtsac.so``.  The
top-level ``mtrl`` package in this repository aliases these modules.
Only the MTSAC / multi-head path is provided; other algorithms and
architectures raise ``NotImplementedError``.
"""
