"""Operators of ``deap.tools`` on the hot path, as device operators.

Crossover: ``cxTwoPoint``, ``cxBlend``, ``cxSimulatedBinaryBounded``; mutation:
``mutFlipBit``, ``mutGaussian``, ``mutPolynomialBounded``; selection: ``selTournament``, ``selRandom``, ``selBest``,
``selWorst``, ``selNSGA2``, ``selTournamentDCD``, ``sortNondominated``
(``emo.assignCrowdingDist``);
migration: ``migRing``; bookkeeping: ``Statistics``, ``MultiStatistics``,
``Logbook``, ``HallOfFame``; initialisation: ``initPopulation``.
"""
from .crossover import cxBlend, cxSimulatedBinaryBounded, cxTwoPoint
from .emo import selNSGA2, selTournamentDCD, sortLogNondominated, sortNondominated
from . import emo
from .init import initPopulation
from .migration import migRing
from .mutation import mutFlipBit, mutGaussian, mutPolynomialBounded
from .selection import selBest, selRandom, selTournament, selWorst
from .support import HallOfFame, Logbook, MultiStatistics, Statistics

__all__ = ["cxTwoPoint", "cxBlend", "cxSimulatedBinaryBounded", "mutFlipBit", "mutGaussian",
           "mutPolynomialBounded", "selTournament", "selRandom",
           "selBest", "selWorst", "selNSGA2", "selTournamentDCD", "sortNondominated", "sortLogNondominated", "migRing", "Statistics",
           "MultiStatistics", "Logbook", "HallOfFame", "initPopulation", "emo"]
