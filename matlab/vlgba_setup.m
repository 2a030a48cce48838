function vlgba_setup()
%VLGBA_SETUP  Put the vlgba MEX gateways and drop-ins before VLG's toolbox/bundle.
%   Run after vlg_setup: addpath(fileparts(mfilename('fullpath')), '-begin').
addpath(fileparts(mfilename('fullpath')), '-begin');
end
