// dropin_predict.hxx -- TEST INFRASTRUCTURE (oracle/Makefile target
// _ref/main_dropin): stands in for the reference's inc/predict.hxx when the
// reference's own main.cxx is compiled against the MI355X library, exactly the
// header swap INTEGRATION.md §1 describes.  Nothing of the reference is
// copied: the build links its other headers where they lie.
#pragma once
#include "nlp/predict.hxx"
