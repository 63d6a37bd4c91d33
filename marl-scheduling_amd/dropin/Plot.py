"""Drop-in ``Plot`` stand-in: plotting is outside this build's hot path.

trainPPO.py imports it with ``from Plot import *`` and only calls the plot
functions when PLOTTING is set; keep the reference's Plot.py on the path
instead of this one to plot results.
"""


def plotFixPricesResult(argsDict):
    raise NotImplementedError("plotting is outside this build's hot path; use the reference's Plot.py")


def plotFreePricesResult(argsDict):
    raise NotImplementedError("plotting is outside this build's hot path; use the reference's Plot.py")
